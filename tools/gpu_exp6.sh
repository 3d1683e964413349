#!/bin/bash
# GPU tests with the Lambert regen default, the screen-tile share table, c5's 3-wave regen variant, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out/exp6; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo pytest=$rc; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c4; do
  timeout -k 10 240 python tools/shard_time.py $c 1 2 4 8 >> $O/shard.jsonl 2>>$O/err.log; rc=$?
  echo shard $c rc=$rc; [ $rc -eq 0 ] || exit $rc
done
cat $O/shard.jsonl
if [ -f opengl_ray_tracing_amd/_variants/libpt_w3.so ]; then
  timeout -k 10 400 python tools/tune.py --variants base w3 --config c5 --frames 30 --warmup 100 --rounds 2 > $O/tune_c5.jsonl 2>>$O/err.log; rc=$?
  echo c5 rc=$rc; tail -1 $O/tune_c5.jsonl; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?; echo bench=$rc; tail -1 $O/bench.log | cut -c1-900
