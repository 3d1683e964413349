#!/bin/bash
# Round-5 evidence on one box: the default bench line, rocprofv3 passes of c4 (c2 and c5 are
# profiles/r5 already), the regen kernel's phases (c2, c5), one rank's share at N = 1 2 4 8
# over the driver's 20-frame window and over 200 frames (c2, c4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_run.sh bench:--steps+20+--warmup+5 || exit 1
cp gpurun_out/bench_step.log gpurun_out/bench_default.log
bash tools/gpu_run.sh profile:r5,c4 phases:c2,c5 shard:c2,20 shard:c2,200 shard:c4,20 shard:c4,200 || exit 1
