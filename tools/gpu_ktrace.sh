#!/bin/bash
# Kernel trace of the bench line (rocprofv3 --kernel-trace) at given frames-in-flight depths.
#   bash tools/gpu_ktrace.sh <config> "<depths>" [steps]   -> gpurun_out/ktrace_<config>_d<depth>/
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=${1:-c2}; DEPTHS=${2:-1 8}; K=${3:-20}
cd /tmp && export TMPDIR=/tmp
for d in $DEPTHS; do
  OUT="$REPO/gpurun_out/ktrace_${CFG}_d$d"; mkdir -p "$OUT"
  PT_PIPE_DEPTH=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
    python3 "$REPO/bench.py" --config $CFG --steps $K --warmup 5 --no-cpu-baseline --no-psnr --no-serial \
    --no-reset > "$OUT/log.txt" 2>&1 || exit $?
  find "$OUT" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
  find "$OUT" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
done
