#!/bin/bash
# Round-4 session V: the camera hit's emission reloaded at the path's end (megakernel MIS) / its
# material index kept instead of the emission (regen kernels), against h4 = the previous commit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -2 gpurun_out/v_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c4 --frames 80 --rounds 4 --variants base h4 > gpurun_out/v_tune_c4.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/v_tune_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c5 --frames 16 --rounds 3 --variants base h4 > gpurun_out/v_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/v_tune_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 80 --rounds 3 --variants base h4 > gpurun_out/v_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/v_tune_c2.log
exit $rc
