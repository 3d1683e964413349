#!/bin/bash
# HIP API time of one rank's share of an N-way split (tools/shard_time.py) under rocprofv3 --hip-trace.
#   bash tools/gpu_api_trace.sh <config> <N>   -> gpurun_out/atrace_<config>_<N>/hip_stats.csv
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=${1:-c2}; N=${2:-8}
OUT="$REPO/gpurun_out/atrace_${CFG}_$N"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --stats -f csv -d "$OUT" -o run -- \
  python3 "$REPO/tools/shard_time.py" $CFG $N > "$OUT/log.txt" 2>&1 || exit $?
find "$OUT" -name '*hip_api_stats.csv' -exec cp {} "$OUT/hip_stats.csv" \;
