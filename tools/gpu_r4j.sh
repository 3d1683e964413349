#!/bin/bash
# Round-4 session J: the regen kernel's phases (PT_PHASE_STATS build) on c5 and c2, then the
# rocprofv3 evidence of the bench line for c2, c4 and c5 (tools/gpu_profile.sh r4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in c5 c2; do
  rm -f "gpurun_out/phases_$c.bin"
  PT_WAVE_TRACE_FILE="gpurun_out/phases_$c.bin" timeout -k 10 300 python -u tools/tune.py --child phases --config "$c" --frames 2 --warmup 0 > "gpurun_out/phases_$c.log" 2>&1; rc=$?
  echo "phases_$c=$rc"; tail -1 "gpurun_out/phases_$c.log"; [ $rc -eq 0 ] || exit $rc
  python tools/wave_trace.py --phases "gpurun_out/phases_$c.bin" | tee "gpurun_out/phases_$c.txt"
done
bash tools/gpu_r4c.sh "${1:-c2 c4 c5}"
