#!/bin/bash
# Round-4 session U: the MIS wide regen kernel as one 1024-thread block per CU with the tree's top
# ~877 nodes in LDS (TOP_BIG, base) against 256-thread blocks with 128 nodes each (bt0): GPU
# tests, then c5 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/u_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -2 gpurun_out/u_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/tune.py --config c5 --frames 16 --rounds 3 --variants base bt0 > gpurun_out/u_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/u_tune_c5.log
exit $rc
