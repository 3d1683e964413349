set -o pipefail
mkdir -p gpurun_out
for c in c2 c4 c5; do
  for f in 0 512 0 512; do
    timeout -k 10 300 python bench.py --config $c --steps 40 --warmup 5 --no-cpu-baseline --no-psnr --flags $f > gpurun_out/ab_${c}_${f}.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${c}_${f}.json')); print('$c flags=$f', d['ms_per_step'], d['config'].get('traversal_tree'))"
  done
done
