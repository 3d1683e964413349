#!/bin/bash
# Round-4 session A3: frames per launch = 2 x N for the screen-tile shares, and repeated bench lines
# at 1 and 2 frames per launch (N = 1) for c2, c4 and c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c2 c4; do
  PT_BATCH_MUL=2 timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shardx2_$c.log" 2>&1; rc=$?
  echo "shardx2_$c=$rc"; grep '^{' "gpurun_out/shardx2_$c.log" | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  bash tools/gpu_batch_sweep.sh "c2 c4" "1 2" 60 || exit $?
  for f in gpurun_out/batch_c2_*.json gpurun_out/batch_c4_*.json; do cp "$f" "${f%.json}_r$r.json"; done
done
bash tools/gpu_batch_sweep.sh "c5" "1 2" 20
