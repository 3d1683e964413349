#!/bin/bash
# Hardware counter passes (each pass its own rocprofv3 run, --pmc only with kernel dispatch
# records) on a short render of config $2 with renderer flags $3 (tools/tune.py child).
# Output: gpurun_out/pmc_<tag>_<cfg>/<pass>/; summarise with tools/pmc_summary.py.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"; CFG="${2:-c2}"; FLAGS="${3:-0}"
OUT="$REPO/gpurun_out/pmc_${TAG}_${CFG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RUN=(python3 "$REPO/tools/tune.py" --child base --config "$CFG" --frames 5 --warmup 16 --flags "$FLAGS" ${MB:+--max-bounce $MB})
PASSES=(
  "A:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "B:SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VMEM"
  "C:TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum"
  "D:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_SMEM SQ_WAVES_LT_64 SQ_INSTS_VSKIPPED SQ_ACTIVE_INST_SCA"
  "E:TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
)
for p in "${PASSES[@]}"; do
  name="${p%%:*}"; ctr="${p#*:}"
  [ -n "$ONLY" ] && [[ "$ONLY" != *"$name"* ]] && continue   # ONLY=AE: a subset of the passes
  timeout -k 10 300 rocprofv3 --pmc $ctr -f csv -d "$OUT/$name" -o run -- "${RUN[@]}" > "$OUT/$name.log" 2>&1; rc=$?
  echo "pass $name=$rc"; [ $rc -eq 0 ] || exit $rc
done
