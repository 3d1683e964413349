#!/bin/bash
# Bench line (as the driver runs it: K steps from an idle GPU) under run-time switches.
#   bash tools/env_sweep.sh "c2 c4" K "ENV=a ENV2=b" "ENV=c" ...   -> gpurun_out/env_sweep.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFGS=$1; K=$2; shift 2
for c in $CFGS; do for e in "$@"; do
  env $e timeout -k 10 120 python bench.py --config $c --steps $K --warmup 5 --no-cpu-baseline \
    --no-psnr --no-serial --no-reset > gpurun_out/env.tmp 2>&1; rc=$?
  [ $rc -eq 0 ] || { cat gpurun_out/env.tmp; exit $rc; }
  python - "$c" "$e" "$K" >> gpurun_out/env_sweep.log <<'PY'
import json, sys
line = [l for l in open("gpurun_out/env.tmp") if l.startswith("{")][-1]
j = json.loads(line)
print(json.dumps({"config": sys.argv[1], "env": sys.argv[2], "steps": int(sys.argv[3]),
                  "ms_per_step": j["ms_per_step"], "value": j["value"]}), flush=True)
PY
  tail -1 gpurun_out/env_sweep.log
done; done
