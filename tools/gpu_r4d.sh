#!/bin/bash
# Round-4 session D: A/B of the megakernel on c5 (FLAG_MEGAKERNEL = 1024: its 3-wave variant),
# of the MIS megakernel at 3 waves per SIMD on c4 (variant mw3), of the whole-tree-in-LDS regen
# kernel on c2 (variant noldstree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/tune.py --variants base --flags 0 1024 --config c5 --frames 20 --rounds 2 > gpurun_out/tune_c5_mega.log 2>&1; rc=$?
echo "c5=$rc"; tail -1 gpurun_out/tune_c5_mega.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tune.py --variants base mw3 --config c4 --frames 60 --rounds 3 > gpurun_out/tune_c4_mw3.log 2>&1; rc=$?
echo "c4=$rc"; tail -1 gpurun_out/tune_c4_mw3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tune.py --variants base noldstree --config c2 --frames 60 --rounds 3 > gpurun_out/tune_c2_lds.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/tune_c2_lds.log
exit $rc
