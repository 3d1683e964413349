#!/bin/bash
# Round-4 session P: a visit's pushes as one push3 (one overflow check) against three push()
# calls (h3 = the previous commit): parity of the 4-wide walks, then c2 / c4 / c5 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -2 gpurun_out/p_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 80 --rounds 3 --variants base h3 > gpurun_out/p_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/p_tune_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c4 --frames 60 --rounds 3 --variants base h3 > gpurun_out/p_tune_c4.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/p_tune_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c5 --frames 12 --rounds 2 --variants base h3 > gpurun_out/p_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/p_tune_c5.log
exit $rc
