#!/bin/bash
# Round-4 session F: the regen kernel's camera-pass shading (main loop / refill loop) against the
# kernel before the shared shading path, on c2 and c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/tune.py --variants base pend0 oldregen --config c2 --frames 60 --rounds 3 > gpurun_out/tune_c2_pend.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/tune_c2_pend.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --variants base pend0 oldregen --config c5 --frames 20 --rounds 2 > gpurun_out/tune_c5_pend.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/tune_c5_pend.log
exit $rc
