#!/bin/bash
# Round-4 session T: 20 frames from an idle GPU (the driver's bench window) with 1 x N and 2 x N
# (default) frames per launch under the round-4 grid shares, c2 and c4, two runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for c in c2 c4; do
    for m in 1 2; do
      PT_SHARD_FRAMES=20 PT_BATCH_MUL=$m timeout -k 10 300 python -u tools/shard_time.py "$c" 1 2 4 8 > "gpurun_out/t_${c}_x${m}_$rep.log" 2>&1; rc=$?
      echo "$c x$m run $rep: $(grep '^{' gpurun_out/t_${c}_x${m}_$rep.log | python3 -c 'import sys,json; print(" ".join(str(json.loads(l)["rank0_ms_per_frame"]) for l in sys.stdin))')"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
