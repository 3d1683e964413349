#!/bin/bash
# Frame-pipeline session: GPU tests, then wall ms per frame of the configs and of one
# rank's share of the screen-tile split (tools/shard_time.py) at pipeline depths
# $DEPTHS. Every GPU step has its own time limit; a crash stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pipe
[ -n "$HWQ" ] && export GPU_MAX_HW_QUEUES=$HWQ
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -2 gpurun_out/pipe/pytest_gpu.log
  ok $rc || exit $rc
fi
for d in ${DEPTHS:-2 3 4}; do
  for c in ${CONFIGS:-c2 c4}; do
    if [ "$d" = probe ]; then unset PT_PIPE_DEPTH; else export PT_PIPE_DEPTH=$d; fi
    timeout -k 10 300 python tools/shard_time.py $c ${WORLDS:-1 2 4 8} > gpurun_out/pipe/shard_${c}_d$d.jsonl 2>gpurun_out/pipe/shard_${c}_d$d.err; rc=$?
    echo "depth=$d $c rc=$rc"; cat gpurun_out/pipe/shard_${c}_d$d.jsonl
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
