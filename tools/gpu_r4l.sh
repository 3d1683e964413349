#!/bin/bash
# Round-4 session L: the regen kernel with the tile's camera-ray results loaded at claim time
# (PT_TILE_PRIM, base) against each lane loading its own (tp0): GPU tests, then c2 and c5 A/B;
# the yield threshold on c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/l_pytest.log 2>&1; rc=$?
echo "pytest=$rc"; tail -3 gpurun_out/l_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 60 --rounds 3 --variants base tp0 > gpurun_out/l_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/l_tune_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c5 --frames 12 --rounds 2 --variants base tp0 > gpurun_out/l_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/l_tune_c5.log; [ $rc -eq 0 ] || exit $rc
# the dynamic ray fetch's yield threshold on c2 (tuned on c5 only: 40)
timeout -k 10 900 python -u tools/tune.py --config c2 --frames 60 --rounds 2 --variants base y24 y32 y48 y56 > gpurun_out/l_yield_c2.log 2>&1; rc=$?
echo "yield=$rc"; tail -1 gpurun_out/l_yield_c2.log
exit $rc
