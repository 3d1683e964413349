#!/bin/bash
# Round-4 session AK: c2 profile and shares with the 4-wave Lambert kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_r4c.sh c2 || exit $?
timeout -k 10 300 python -u tools/shard_time.py c2 1 2 4 8 > gpurun_out/ak200_c2.log 2>&1 || exit 1
PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py c2 1 2 4 8 > gpurun_out/ak20_c2.log 2>&1 || exit 1
echo "c2 200f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ak200_c2.log | cut -d' ' -f2 | tr '\n' ' ') 20f: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ak20_c2.log | cut -d' ' -f2 | tr '\n' ' ')"
