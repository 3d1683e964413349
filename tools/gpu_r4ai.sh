#!/bin/bash
# Round-4 session AI: c5 frames per launch (1 default / 2) and frames in flight (3 / 4 default / 6)
# after the register trims, 100 frames at N = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { timeout -k 10 300 python -u tools/shard_time.py c5 1 > "gpurun_out/ai_$1.log" 2>&1 || exit 1; echo "$1: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ai_$1.log)"; }
export PT_SHARD_FRAMES=100
run base
PT_BATCH=2 run b2
PT_PIPE_DEPTH=3 run d3
PT_PIPE_DEPTH=6 run d6
run base2
