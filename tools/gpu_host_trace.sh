#!/bin/bash
# HIP API calls beside the kernels of one rank's share of an N-way split (tools/shard_time.py):
# where the host time of a pt_render_frames_async call and its gather goes.
#   bash tools/gpu_host_trace.sh <config> <N> [frames]  -> gpurun_out/htrace_<config>_<N>/{kernel,hip_api}_trace.csv
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=${1:-c2}; N=${2:-8}; F=${3:-20}
OUT="$REPO/gpurun_out/htrace_${CFG}_$N"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PT_SHARD_FRAMES=$F timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d "$OUT" -o run -- \
  python3 "$REPO/tools/shard_time.py" $CFG $N > "$OUT/log.txt" 2>&1 || exit $?
find "$OUT" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
find "$OUT" -name '*hip_api_trace.csv' -exec cp {} "$OUT/hip_api_trace.csv" \;
