set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for c in c2 c3 c4; do
timeout -k 10 400 python tools/tune.py --variants base prev --config $c --rounds 3 --frames 40 > gpurun_out/tune_$c.log 2>&1 || exit $?
done
timeout -k 10 400 python tools/tune.py --variants base prev --config c5 --rounds 1 --frames 10 > gpurun_out/tune_c5.log 2>&1 || exit $?
