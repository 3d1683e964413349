#!/bin/bash
# Round-4 session M: the LDS tree at a 7-float4 stride (one address, immediate offsets) against
# the rotated 8-float4 layout (h2 = the previous commit): GPU tests, then c2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -3 gpurun_out/m_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/tune.py --config c2 --frames 80 --rounds 4 --variants base h2 > gpurun_out/m_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/m_tune_c2.log
exit $rc
