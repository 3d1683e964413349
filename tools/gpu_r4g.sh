#!/bin/bash
# Round-4 session G: c5's screen-tile shares (frame batches), and c4's at 2 x N frames per launch
# with the 3-wave MIS megakernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/shard_time.py c5 1 2 4 8 > gpurun_out/shard12_c5.log 2>&1; rc=$?
echo "shard_c5=$rc"; grep '^{' gpurun_out/shard12_c5.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
for c in c2 c4; do
  timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shard12b_$c.log" 2>&1; rc=$?
  echo "shard_$c=$rc"; grep '^{' "gpurun_out/shard12b_$c.log" | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
