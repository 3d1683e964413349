#!/bin/bash
# Round-4 session A: smoke, GPU tests and the bench (tools/gpu_check.sh), one rank's share of the
# screen-tile split with frame batches (tools/shard_time.py), and the whole-tree-in-LDS regen
# kernel against the variant without it (tools/tune.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
for c in c2 c4; do
  timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shard_$c.log" 2>&1; rc=$?
  echo "shard_$c=$rc"; cat "gpurun_out/shard_$c.log" | grep '^{' | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u tools/tune.py --variants base noldstree --config c2 --rounds 3 > gpurun_out/tune_ldstree.log 2>&1; rc=$?
echo "tune=$rc"; tail -4 gpurun_out/tune_ldstree.log
exit $rc
