#!/bin/bash
# Round-4 session AB: final shard times, bench line and the regen kernel's phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r4q.sh || exit $?
for c in c2 c5; do
  rm -f "gpurun_out/phases_$c.bin"
  PT_WAVE_TRACE_FILE="gpurun_out/phases_$c.bin" timeout -k 10 300 python -u tools/tune.py --child phases --config "$c" --frames 2 --warmup 0 > "gpurun_out/phases_$c.log" 2>&1; rc=$?
  echo "phases_$c=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/wave_trace.py --phases "gpurun_out/phases_$c.bin" | tee "gpurun_out/phases_$c.txt"
done
