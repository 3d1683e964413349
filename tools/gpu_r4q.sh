#!/bin/bash
# Round-4 session Q: final screen-tile shares (200 frames, and 20 frames from an idle GPU) for c2
# and c4, c5 N = 1 / 8, and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c2 c4; do
  timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/q200_$c.log" 2>&1; rc=$?
  echo "q200_$c=$rc"; grep '^{' "gpurun_out/q200_$c.log" | cut -c1-110; [ $rc -eq 0 ] || exit $rc
  PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/q20_$c.log" 2>&1; rc=$?
  echo "q20_$c=$rc"; grep '^{' "gpurun_out/q20_$c.log" | cut -c1-110; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u tools/shard_time.py c5 1 8 > gpurun_out/q200_c5.log 2>&1; rc=$?
echo "q200_c5=$rc"; grep '^{' gpurun_out/q200_c5.log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/q_bench.log 2>&1; rc=$?
echo "bench=$rc"; tail -c 400 gpurun_out/q_bench.log
exit $rc
