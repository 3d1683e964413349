#!/bin/bash
# Round-4 session L: GPU tests; A/B of base (the claimed tile's camera-ray results read from
# neighbour lanes, PT_TILE_PRIM, + the walks' winners' triangle indices read from the pair
# records) against head (the tile prefetch alone) and tp0 (neither); the yield threshold on c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/l_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -3 gpurun_out/l_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 60 --rounds 3 --variants base head tp0 > gpurun_out/l_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/l_tune_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c4 --frames 60 --rounds 3 --variants base head > gpurun_out/l_tune_c4.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/l_tune_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c5 --frames 12 --rounds 2 --variants base head tp0 > gpurun_out/l_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/l_tune_c5.log; [ $rc -eq 0 ] || exit $rc
# the dynamic ray fetch's yield threshold on c2 (tuned on c5 only: 40); variants built before the pair ids
timeout -k 10 900 python -u tools/tune.py --config c2 --frames 60 --rounds 2 --variants head y24 y32 y48 y56 > gpurun_out/l_yield_c2.log 2>&1; rc=$?
echo "yield=$rc"; tail -1 gpurun_out/l_yield_c2.log
exit $rc
