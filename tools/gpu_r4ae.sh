#!/bin/bash
# Round-4 session AE: frames per launch at N = 1 for c2 and c4 after the kernel changes
# (PT_BATCH 1 / 2 (default) / 3 / 4), over 200 frames and over 20 frames from an idle GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c2 c4; do
  for b in 1 2 3 4; do
    PT_BATCH=$b timeout -k 10 300 python -u tools/shard_time.py "$c" 1 > "gpurun_out/ae_${c}_b$b.log" 2>&1; rc=$?
    PT_SHARD_FRAMES=20 PT_BATCH=$b timeout -k 10 300 python -u tools/shard_time.py "$c" 1 > "gpurun_out/ae20_${c}_b$b.log" 2>&1; rc2=$?
    echo "$c batch $b: 200f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ae_${c}_b$b.log) 20f $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ae20_${c}_b$b.log)"
    [ $rc -eq 0 ] && [ $rc2 -eq 0 ] || exit 1
  done
done
