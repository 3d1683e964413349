#!/bin/bash
# Round-4 session AH: megakernel frames per launch max(8, 4 x N): GPU tests, c4 shares, c3 N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ah_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -2 gpurun_out/ah_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_time.py c4 1 2 4 8 > gpurun_out/ah200_c4.log 2>&1 || exit 1
PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py c4 1 2 4 8 > gpurun_out/ah20_c4.log 2>&1 || exit 1
echo "c4 200f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ah200_c4.log | cut -d' ' -f2 | tr '\n' ' ') 20f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ah20_c4.log | cut -d' ' -f2 | tr '\n' ' ')"
for b in 0 4; do
  PT_BATCH=$b timeout -k 10 300 python -u tools/shard_time.py c4 1 > "gpurun_out/ah_c4_b$b.log" 2>&1 || exit 1
  PT_SHARD_FRAMES=20 PT_BATCH=$b timeout -k 10 300 python -u tools/shard_time.py c4 1 > "gpurun_out/ah20_c4_b$b.log" 2>&1 || exit 1
  echo "c4 N=1 batch $b (0 = default 8): 200f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ah_c4_b$b.log) 20f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ah20_c4_b$b.log)"
done
PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py c3 1 > gpurun_out/ah20_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/shard_time.py c3 1 > gpurun_out/ah200_c3.log 2>&1 || exit 1
echo "c3 N=1: 200f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ah200_c3.log) 20f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ah20_c3.log)"
