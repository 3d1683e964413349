#!/bin/bash
# Round-5 evidence on one box: the default bench line (as the driver runs it, CPU baseline
# included), the regen kernel's phases (c2, c5), one rank's share at N = 1 2 4 8 over the driver's
# 20-frame window and over 200 frames (c2, c4). The rocprofv3 passes: tools/gpu_profile.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
tail -c 300 gpurun_out/bench_default.log
bash tools/gpu_run.sh phases:c2,c5 shard:c2,20 shard:c2,200 shard:c4,20 shard:c4,200 || exit 1
