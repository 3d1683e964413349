#!/bin/bash
# Round-4 session E: the GPU suite, then bench lines (default frames per launch) for c2, c4, c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  bash tools/gpu_batch_sweep.sh "c2 c4" "0" 60 || exit $?
  bash tools/gpu_batch_sweep.sh "c5" "0" 20 || exit $?
done
