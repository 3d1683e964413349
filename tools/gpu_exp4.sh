#!/bin/bash
# GPU tests, then the running mean inside the frame kernels (default) vs mixKernel per frame
# (PT_KERNEL_MIX=0) for one rank's share of the screen-tile split, then the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out/exp4; mkdir -p $O; cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo pytest=$rc; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for km in ${MIXES:-1 0 1}; do for c in ${CONFIGS:-c2 c4}; do
  echo "kernel_mix=$km" >> $O/mix.jsonl
  PT_KERNEL_MIX=$km timeout -k 10 240 python tools/shard_time.py $c 1 2 4 8 >> $O/mix.jsonl 2>>$O/err.log; rc=$?
  echo kernel_mix=$km $c rc=$rc; [ $rc -eq 0 ] || exit $rc
done; done
cat $O/mix.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo bench=$rc; tail -1 $O/bench.log | cut -c1-600
