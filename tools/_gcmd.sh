set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --dist-backend gloo --same-device > gpurun_out/bench_n2.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --dist-backend gloo --same-device --shard tiles > gpurun_out/bench_n2t.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || exit $?
