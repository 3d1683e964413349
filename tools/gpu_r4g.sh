#!/bin/bash
# Round-4 session G: screen-tile shares with the current defaults (c2, c4, c5), and over 20 frames
# from an idle GPU (the driver's bench line) at 1 x N and 2 x N frames per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c2 c4; do
  timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shard12b_$c.log" 2>&1; rc=$?
  echo "shard_$c=$rc"; grep '^{' "gpurun_out/shard12b_$c.log" | cut -c1-120; [ $rc -eq 0 ] || exit $rc
  for m in 1 2; do
    PT_SHARD_FRAMES=20 PT_BATCH_MUL=$m timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shard20_${c}_x$m.log" 2>&1; rc=$?
    echo "shard20_${c}_x$m=$rc"; grep '^{' "gpurun_out/shard20_${c}_x$m.log" | cut -c1-120; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 600 python -u tools/shard_time.py c5 1 8 > gpurun_out/shard12_c5.log 2>&1; rc=$?
echo "shard_c5=$rc"; grep '^{' gpurun_out/shard12_c5.log | cut -c1-120
exit $rc
