#!/bin/bash
# Round-4 session K: the wavefront pipeline with the 4-wide trace kernel (wfTrace4Kernel) --
# parity, then c5 wall ms per frame against the regen kernel (pipelined and serial), and a
# kernel trace of its stages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "frame_kernels_agree" > gpurun_out/k_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -3 gpurun_out/k_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/tune.py --config c5 --frames 10 --rounds 2 --flags 0 8 128 > gpurun_out/k_tune_c5.log 2>&1; rc=$?
echo "tune=$rc"; cat gpurun_out/k_tune_c5.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/k_wf" -o run -- python3 "$GRAFT_REPO_ROOT/tools/tune.py" --child base --config c5 --frames 3 --warmup 0 --flags 8 > "$GRAFT_REPO_ROOT/gpurun_out/k_wf.log" 2>&1; rc=$?
echo "wf_trace=$rc"; find "$GRAFT_REPO_ROOT/gpurun_out/k_wf" -name "*kernel_stats.csv" -exec head -12 {} \; | cut -c1-200
exit $rc
