# A/B of render flags: bash tools/ab_flags.sh <config> <flags...>  (one bench line per flag value)
set -o pipefail
mkdir -p gpurun_out
c=$1; shift
for f in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-psnr --flags $f > gpurun_out/ab_${c}_${f}.json 2>gpurun_out/ab_${c}_${f}.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ab_${c}_${f}.json')); print('$c flags=$f', d['ms_per_step'], d['roofline'].get('kernel_ms'), d['config'].get('traversal_tree'), d['config'].get('waves_per_simd'))"
done
