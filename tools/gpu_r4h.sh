#!/bin/bash
# Round-4 session H: grid share from the launches actually in flight (base) vs 150 % / depth
# (the fixedshare tuning build), over 20 frames from an idle GPU and over 200 frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base fixedshare; do
    for c in c2 c4; do
      pv=""; [ "$v" = base ] || pv=$v
      PT_VARIANT=$pv PT_SHARD_FRAMES=20 timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/h20_${v}_${c}_$rep.log" 2>&1; rc=$?
      echo "h20_${v}_${c}_$rep=$rc"; grep '^{' "gpurun_out/h20_${v}_${c}_$rep.log" | cut -c1-100; [ $rc -eq 0 ] || exit $rc
    done
  done
done
for c in c2 c4; do
  timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/h200_$c.log" 2>&1; rc=$?
  echo "h200_$c=$rc"; grep '^{' "gpurun_out/h200_$c.log" | cut -c1-100; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py > gpurun_out/h_bench.log 2>&1; rc=$?
echo "bench=$rc"; tail -c 600 gpurun_out/h_bench.log
exit $rc
