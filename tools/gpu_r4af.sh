#!/bin/bash
# Round-4 session AF: c4 (megakernel) frames per launch: 2 x N (default) against 4 x N at
# N = 1 / 2 / 4 / 8, over 200 frames and 20 frames from idle; batches of 6 and 8 at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 2 4; do
  PT_BATCH_MUL=$m timeout -k 10 300 python -u tools/shard_time.py c4 1 2 4 8 > "gpurun_out/af_c4_x$m.log" 2>&1 || exit 1
  PT_SHARD_FRAMES=20 PT_BATCH_MUL=$m timeout -k 10 300 python -u tools/shard_time.py c4 1 2 4 8 > "gpurun_out/af20_c4_x$m.log" 2>&1 || exit 1
  echo "c4 x$m 200f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/af_c4_x$m.log | cut -d' ' -f2 | tr '\n' ' ') 20f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/af20_c4_x$m.log | cut -d' ' -f2 | tr '\n' ' ')"
done
for b in 6 8; do
  PT_BATCH=$b timeout -k 10 300 python -u tools/shard_time.py c4 1 > "gpurun_out/af_c4_b$b.log" 2>&1 || exit 1
  PT_SHARD_FRAMES=20 PT_BATCH=$b timeout -k 10 300 python -u tools/shard_time.py c4 1 > "gpurun_out/af20_c4_b$b.log" 2>&1 || exit 1
  echo "c4 batch $b: 200f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/af_c4_b$b.log) 20f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/af20_c4_b$b.log)"
done
