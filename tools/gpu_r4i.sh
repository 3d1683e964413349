#!/bin/bash
# Round-4 session I: the regen kernel's phases (PT_PHASE_STATS build) on c5 and c2, after the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
for c in c5 c2; do
  rm -f "gpurun_out/phases_$c.bin"
  PT_WAVE_TRACE_FILE="gpurun_out/phases_$c.bin" timeout -k 10 300 python -u tools/tune.py --child phases --config "$c" --frames 2 --warmup 0 > "gpurun_out/phases_$c.log" 2>&1; rc=$?
  echo "phases_$c=$rc"; tail -2 "gpurun_out/phases_$c.log"; [ $rc -eq 0 ] || exit $rc
  python tools/wave_trace.py --phases "gpurun_out/phases_$c.bin" | tee "gpurun_out/phases_$c.txt"
done
