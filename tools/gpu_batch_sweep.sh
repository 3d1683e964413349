#!/bin/bash
# Bench lines (N = 1) at several frames-per-launch batches (pt_config.frame_batch) per config.
#   bash tools/gpu_batch_sweep.sh "<configs>" "<batches>" [steps]  -> gpurun_out/batch_<cfg>_<b>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${3:-40}
for c in $1; do
  for b in $2; do
    timeout -k 10 300 python bench.py --config "$c" --steps "$STEPS" --warmup 5 --batch "$b" --no-cpu-baseline \
      --no-psnr --no-serial --no-reset > "gpurun_out/batch_${c}_${b}.json" 2> "gpurun_out/batch_${c}_${b}.err"; rc=$?
    echo "$c batch $b rc=$rc $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['ms_per_step'], d['value'])" "gpurun_out/batch_${c}_${b}.json" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
