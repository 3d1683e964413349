#!/bin/bash
# Round-4 session AG: GPU tests with 4 x tile_world frames per megakernel launch, then c4 shares
# and c3 at N = 1 against 2 x (PT_BATCH_MUL=2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ag_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -2 gpurun_out/ag_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_time.py c4 1 2 4 8 > gpurun_out/ag200_c4.log 2>&1 || exit 1
PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py c4 1 2 4 8 > gpurun_out/ag20_c4.log 2>&1 || exit 1
echo "c4 200f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ag200_c4.log | cut -d' ' -f2 | tr '\n' ' ') 20f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ag20_c4.log | cut -d' ' -f2 | tr '\n' ' ')"
for m in 0 2; do
  PT_BATCH_MUL=$m timeout -k 10 300 python -u tools/shard_time.py c3 1 > "gpurun_out/ag_c3_x$m.log" 2>&1 || exit 1
  PT_SHARD_FRAMES=20 PT_BATCH_MUL=$m timeout -k 10 300 python -u tools/shard_time.py c3 1 > "gpurun_out/ag20_c3_x$m.log" 2>&1 || exit 1
  echo "c3 mul $m: 200f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ag_c3_x$m.log) 20f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ag20_c3_x$m.log)"
done
