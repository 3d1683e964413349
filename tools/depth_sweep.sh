#!/bin/bash
# Frames-in-flight sweep of the bench line as the driver runs it (K steps from an idle
# GPU, fill and drain included): PT_PIPE_DEPTH x config, then the same at K=100.
#   bash tools/depth_sweep.sh "c2 c4" "1 2 3 4 8" [K]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=${1:-c2 c4}; DEPTHS=${2:-1 2 3 4 8}; K=${3:-20}
for c in $CFGS; do for d in $DEPTHS; do
  PT_PIPE_DEPTH=$d timeout -k 10 120 python bench.py --config $c --steps $K --warmup 5 --no-cpu-baseline \
    --no-psnr --no-serial --no-reset > gpurun_out/depth.tmp 2>&1; rc=$?
  [ $rc -eq 0 ] || { cat gpurun_out/depth.tmp; exit $rc; }
  python - "$c" "$d" "$K" >> gpurun_out/depth_sweep.log <<'PY'
import json, sys
line = [l for l in open("gpurun_out/depth.tmp") if l.startswith("{")][-1]
j = json.loads(line)
print(json.dumps({"config": sys.argv[1], "depth": int(sys.argv[2]), "steps": int(sys.argv[3]),
                  "ms_per_step": j["ms_per_step"], "value": j["value"]}), flush=True)
PY
  tail -1 gpurun_out/depth_sweep.log
done; done
