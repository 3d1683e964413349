#!/bin/bash
# One GPU session: smoke -> gpu tests -> short bench. Each GPU step has its own
# time limit; a crash/timeout (exit >= 2 other than pytest's 1) stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"
ok $rc || exit $rc
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
tail -3 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline} > gpurun_out/bench.log 2>&1; rc=$?; echo "bench=$rc"
tail -c 600 gpurun_out/bench.log
exit $rc
