#!/bin/bash
# Round-4 session AD: the tile camera-ray prefetch for the MIS regen kernel too (tpm), now that
# it barely spills.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune.py --config c5 --frames 16 --rounds 3 --variants base tpm > gpurun_out/ad_tpm_c5.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/ad_tpm_c5.log
exit $rc
