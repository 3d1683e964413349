#!/bin/bash
# Round-4 session AC: the dynamic ray fetch's yield threshold again after the register trims
# (32 / 40 = base / 48) on c5 and c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune.py --config c5 --frames 16 --rounds 3 --variants base y32 y48 > gpurun_out/ac_yield_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/ac_yield_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 80 --rounds 3 --variants base y32 y48 > gpurun_out/ac_yield_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/ac_yield_c2.log
exit $rc
