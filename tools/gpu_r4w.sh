#!/bin/bash
# Round-4 session W: the 4-wide walks' slab FMAs as scalar v_fma_f32 with the ray held as three
# (1/d, -o/d) pairs (ss: six VGPRs fewer, twelve more VALU per visit) against packed FMAs with
# broadcast pairs (base): GPU tests of the ss build's kernels are run via tune parity only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/tune.py --config c4 --frames 80 --rounds 4 --variants base ss > gpurun_out/w_tune_c4.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/w_tune_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c5 --frames 16 --rounds 3 --variants base ss > gpurun_out/w_tune_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/w_tune_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c2 --frames 80 --rounds 3 --variants base ss > gpurun_out/w_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/w_tune_c2.log
exit $rc
