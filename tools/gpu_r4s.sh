#!/bin/bash
# Round-4 session S: L2 behaviour of the wavefront trace kernel (wfTrace4Kernel) against the regen
# kernel on c5 -- one --pmc pass each over two frames.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$REPO/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for f in 8 0; do
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -f csv -d "$REPO/gpurun_out/s_f$f" -o run -- python3 "$REPO/tools/tune.py" --child base --config c5 --frames 2 --warmup 0 --flags $f > "$REPO/gpurun_out/s_f$f.log" 2>&1; rc=$?
  echo "flags $f: $rc"; [ $rc -eq 0 ] || exit $rc
done
