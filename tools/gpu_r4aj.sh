#!/bin/bash
# Round-4 session AJ: the Lambert LDS-tree regen kernel at 4 waves per SIMD (u4: 3 VGPRs spilled
# since the scalar pair test) against 3 (base), five rounds on c2, and the 20-frame window.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune.py --config c2 --frames 100 --rounds 5 --variants base u4 > gpurun_out/aj_tune_c2.log 2>&1; rc=$?
echo "c2=$rc"; tail -1 gpurun_out/aj_tune_c2.log; [ $rc -eq 0 ] || exit $rc
for v in "" u4; do
  PT_VARIANT=$v PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py c2 1 2 4 8 > "gpurun_out/aj20_c2_${v:-base}.log" 2>&1 || exit 1
  echo "20f ${v:-base}: $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/aj20_c2_${v:-base}.log | cut -d' ' -f2 | tr '\n' ' ')"
done
