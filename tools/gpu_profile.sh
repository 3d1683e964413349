#!/bin/bash
# rocprofv3 evidence for the bench kernel: kernel trace + stats, then HBM
# traffic counters in their own passes (FETCH_SIZE and WRITE_SIZE cannot share
# a pass on gfx950). Output under gpurun_out/prof_<tag>/.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"
CFG="${2:-c2}"
OUT="$REPO/gpurun_out/prof_${TAG}_${CFG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=(python3 "$REPO/bench.py" --config "$CFG" --steps 30 --warmup 5 --no-cpu-baseline)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- "${BENCH[@]}" > "$OUT/trace.log" 2>&1; rc=$?
echo "trace=$rc"; [ $rc -eq 0 ] || exit $rc
BENCH5=(python3 "$REPO/bench.py" --config "$CFG" --steps 5 --warmup 2 --no-cpu-baseline)
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- "${BENCH5[@]}" > "$OUT/fetch.log" 2>&1; rc=$?
echo "fetch=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- "${BENCH5[@]}" > "$OUT/write.log" 2>&1; rc=$?
echo "write=$rc"
exit $rc
