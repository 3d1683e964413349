set -o pipefail
for b in 6 8 12 16; do bash tools/gpu_run.sh bench:--steps+20+--warmup+5+--no-cpu-baseline+--no-psnr+--no-serial+--no-reset+--batch+$b || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log; done
for b in 4 8 16; do bash tools/gpu_run.sh bench:--config+c4+--steps+20+--warmup+5+--no-cpu-baseline+--no-psnr+--no-serial+--no-reset+--batch+$b || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log; done
for b in 1 2; do bash tools/gpu_run.sh bench:--config+c5+--steps+10+--warmup+2+--no-cpu-baseline+--no-psnr+--no-serial+--no-reset+--batch+$b || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_step.log; done
for m in 2 4 8; do PT_BATCH_MUL=$m bash tools/gpu_run.sh shard:c2,20 || exit 1; done
