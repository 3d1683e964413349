#!/bin/bash
# Round-4 session Y: the leaf pair test in scalar VALU (sp: no broadcast pairs of o and d held
# across the walks) against packed (base, scalar slab FMAs already); with the Lambert LDS-tree
# kernel at 4 waves (sp4) and the MIS wide kernel at 3 (sp3m).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 80 --rounds 3 --variants base sp sp4 > gpurun_out/y_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/y_tune_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c4 --frames 80 --rounds 3 --variants base sp > gpurun_out/y_tune_c4.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/y_tune_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/tune.py --config c5 --frames 16 --rounds 3 --variants base sp sp3m > gpurun_out/y_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/y_tune_c5.log
exit $rc
