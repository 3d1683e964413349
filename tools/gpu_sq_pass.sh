#!/bin/bash
# Where a frame kernel's wave-cycles go (rocprofv3 --pmc, one pass of SQ counters over the bench's
# pipelined frames of config $1): waves, wave-cycles, cycles waiting on anything / on instructions,
# active instruction cycles by kind.   bash tools/gpu_sq_pass.sh c2   -> gpurun_out/sq_c2/
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=${1:-c2}
OUT="$REPO/gpurun_out/sq_$CFG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -f csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --config $CFG --steps 16 --warmup 2 --no-cpu-baseline --no-psnr --no-reset --no-serial > "$OUT/log.txt" 2>&1
