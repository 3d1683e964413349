#!/bin/bash
# Kernel trace of one rank's share of an N-way screen-tile split (tools/shard_time.py).
#   bash tools/gpu_shard_trace.sh <config> <N> [frames [tag]]  -> gpurun_out/strace_<config>_<N>[_tag]/kernel_trace.csv
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=${1:-c2}; N=${2:-8}; F=${3:-200}; TAG=${4:+_$4}
OUT="$REPO/gpurun_out/strace_${CFG}_$N$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PT_SHARD_FRAMES=$F timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
  python3 "$REPO/tools/shard_time.py" $CFG $N > "$OUT/log.txt" 2>&1 || exit $?
find "$OUT" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
find "$OUT" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
