#!/bin/bash
# Round-4 session A2 (12 hardware queues, as the bench): the screen-tile share with frame batches,
# the whole-tree-in-LDS A/B, and bench lines at 1 / 2 / 4 frames per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c2 c4; do
  timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shard12_$c.log" 2>&1; rc=$?
  echo "shard_$c=$rc"; grep '^{' "gpurun_out/shard12_$c.log" | cut -c1-150; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u tools/tune.py --variants base noldstree --config c2 --rounds 3 > gpurun_out/tune_ldstree12.log 2>&1; rc=$?
echo "tune=$rc"; tail -1 gpurun_out/tune_ldstree12.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_batch_sweep.sh "c2 c4" "1 2 4" 60
