#!/bin/bash
# Round-4 session Z: small MIS / Disney scenes on the wide regen kernel (ra: every integrator on
# the path-regeneration kernel) against the megakernel (base), now that the MIS kernels barely spill.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/tune.py --config c4 --frames 80 --rounds 3 --variants base ra > gpurun_out/z_tune_c4.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/z_tune_c4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/tune.py --config c3 --frames 80 --rounds 3 --variants base ra > gpurun_out/z_tune_c3.log 2>&1; rc=$?
echo "c3=$rc"; tail -1 gpurun_out/z_tune_c3.log
exit $rc
