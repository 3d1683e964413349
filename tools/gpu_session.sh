#!/bin/bash
# One GPU session: tools/gpu_check.sh (smoke, gpu tests, bench), then one rank's
# share of the screen-tile split for each config named (tools/shard_time.py).
#   bash tools/gpu_session.sh [config ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
for c in "$@"; do
  timeout -k 10 240 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/shard_$c.log" 2>&1; rc=$?
  echo "shard_$c=$rc"; [ $rc -eq 0 ] || exit $rc
done
