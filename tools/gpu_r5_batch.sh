#!/bin/bash
# Round-5 A/B: the 32-frame batch cap (variant mb32) on c2's shares and c4; c4 on the regen kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_run.sh shard:c2,20 shard:c2,20,mb32 || exit 1
for v in "" mb32; do
  PT_VARIANT=$v bash tools/gpu_run.sh bench:--config+c4+--steps+20+--warmup+5+--no-cpu-baseline+--no-psnr+--no-serial+--no-reset || exit 1
  echo "c4 ${v:-base}: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log)"
done
bash tools/gpu_run.sh bench:--config+c4+--steps+20+--warmup+5+--no-cpu-baseline+--no-psnr+--no-serial+--no-reset+--flags+16 || exit 1
echo "c4 regen: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log)"
