#!/bin/bash
# Round-4 session O: the uniform integrators' LDS-tree regen kernel at 4 waves per SIMD (u4:
# one 1024-thread block per CU, 76 VGPRs spilled) against 3 (base).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune.py --config c2 --frames 80 --rounds 3 --variants base u4 > gpurun_out/o_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/o_tune_c2.log
exit $rc
