#!/bin/bash
# Per-kernel time breakdown of one renderer configuration (rocprofv3 kernel trace).
# usage: gpu_kprof.sh <tag> <config> <flags> [variant]
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; CFG="$2"; FLAGS="${3:-0}"; VAR="${4:-base}"
OUT="$REPO/gpurun_out/kprof_${TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
  python3 "$REPO/tools/tune.py" --child "$VAR" --config "$CFG" --frames 10 --warmup 2 --flags "$FLAGS" > "$OUT/log.txt" 2>&1
