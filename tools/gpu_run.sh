#!/bin/bash
# One GPU session as a list of named steps, each under its own time limit; the first step that
# fails ends the session (no retries). Replaces round 4's one-off gpu_r4*.sh session scripts.
#
#   bash tools/gpu_run.sh STEP[:ARG,ARG...] ...
#
# Steps (output under gpurun_out/):
#   check                       smoke, the GPU suite, a short bench (tools/gpu_check.sh)
#   phases:CFG[,CFG...]         the regen kernel's phase statistics (tuning build "phases":
#                               PT_WAVE_TRACE=1,PT_PHASE_STATS=1) -> phases_CFG.txt
#   ta:CFG                      texture-path busy (TA/TD) over serially issued frames -> ta_CFG/
#   profile:TAG,CFG             rocprofv3 kernel trace + counter passes (tools/gpu_profile.sh)
#   shard:CFG[,FRAMES[,VAR]]    one rank's share of the N = 1 2 4 8 split (tools/shard_time.py)
#   tune:CFG,FRAMES,ROUNDS,V... A/B of tuning builds (tools/tune.py)
#   bench[:ARGS]                bench.py with ARGS (spaces as '+'), default --steps 20 --warmup 5
#   pytest:EXPR                 the GPU suite restricted to -k EXPR
#   sq:CFG                      where the bench kernels' wave-cycles go (tools/gpu_sq_pass.sh)
#   attr:CFG,VARIANT...         DRAM-side bytes per frame per build (tools/gpu_attr.sh; tools/attr.py)
#   evidence                    the default bench line (as the driver runs it), phases of c2/c5,
#                               shares of c2/c4 over 20 and 200 frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name="${1%%:*}" arg=""
  [[ "$1" == *:* ]] && arg="${1#*:}"
  IFS=',' read -r -a A <<< "$arg"
  case "$name" in
    check) bash tools/gpu_check.sh ;;
    phases)
      for c in "${A[@]}"; do
        rm -f "gpurun_out/phases_$c.bin"
        PT_WAVE_TRACE_FILE="gpurun_out/phases_$c.bin" timeout -k 10 300 python -u tools/tune.py --child phases \
          --config "$c" --frames 2 --warmup 0 > "gpurun_out/phases_$c.log" 2>&1 || return $?
        python tools/wave_trace.py --phases "gpurun_out/phases_$c.bin" | tee "gpurun_out/phases_$c.txt" || return $?
      done ;;
    ta) bash tools/gpu_ta_pass.sh "${A[0]:-c2}" ;;
    profile) bash tools/gpu_profile.sh "${A[0]:-r5}" "${A[1]:-c2}" ;;
    shard)
      local log="gpurun_out/shard_${A[0]}_${A[1]:-200}_${A[2]:-base}.log"
      PT_VARIANT="${A[2]:-}" PT_SHARD_FRAMES="${A[1]:-200}" timeout -k 10 300 python -u tools/shard_time.py "${A[0]}" 1 2 4 8 \
        > "$log" 2>&1 || return $?
      echo "$log: $(grep -o '"rank0_ms_per_frame": [0-9.]*' "$log" | cut -d' ' -f2 | tr '\n' ' ')" ;;
    tune)
      local log="gpurun_out/tune_${A[0]}_$(IFS=_; echo "${A[*]:3}").log"
      timeout -k 10 900 python -u tools/tune.py --config "${A[0]}" --frames "${A[1]}" --rounds "${A[2]}" \
        --variants "${A[@]:3}" > "$log" 2>&1 || return $?
      tail -1 "$log" ;;
    bench)
      local args="${arg//+/ }"
      timeout -k 10 600 python bench.py ${args:---steps 20 --warmup 5} > gpurun_out/bench_step.log 2>&1 || return $?
      tail -c 800 gpurun_out/bench_step.log ;;
    pytest)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$arg" \
        > "gpurun_out/pytest_k.log" 2>&1 || return $?
      tail -3 gpurun_out/pytest_k.log ;;
    sq) bash tools/gpu_sq_pass.sh "${A[0]:-c2}" ;;
    attr) bash tools/gpu_attr.sh "${A[@]}" ;;
    evidence)
      timeout -k 10 900 python bench.py > gpurun_out/bench_default.log 2>&1 || return $?
      tail -c 300 gpurun_out/bench_default.log
      for s2 in phases:c2,c5 shard:c2,20 shard:c2,200 shard:c4,20 shard:c4,200; do step "$s2" || return $?; done ;;
    *) echo "unknown step $name"; return 2 ;;
  esac
}
for s in "$@"; do
  step "$s"; rc=$?
  echo "step $s rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
