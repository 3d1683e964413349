#!/bin/bash
# Texture-path occupancy of the bench kernel (one rocprofv3 --pmc pass over serially issued frames):
# TA / TD busy cycles summed over the CUs, with GRBM_GUI_ACTIVE for the window.
#   bash tools/gpu_ta_pass.sh <config>   -> gpurun_out/ta_<config>/
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=${1:-c2}
OUT="$REPO/gpurun_out/ta_$CFG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -f csv -d "$OUT" -o run -- \
  python3 "$REPO/bench.py" --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-psnr --no-reset --no-serial \
  --flags 128 > "$OUT/log.txt" 2>&1
