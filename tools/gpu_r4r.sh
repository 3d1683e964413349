#!/bin/bash
# Round-4 session R: frames in flight (PT_PIPE_DEPTH) under the round-4 grid shares and batches:
# c5 at 2 / 3 / 4 / 6, c2 at 4 / 6 / 8 (defaults: c5 4, c2 6).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 4 2 3 6; do
  PT_PIPE_DEPTH=$d timeout -k 10 300 python -u tools/tune.py --config c5 --frames 16 --rounds 2 > "gpurun_out/r_c5_d$d.log" 2>&1; rc=$?
  echo "c5 depth $d: $(tail -1 gpurun_out/r_c5_d$d.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
for d in 6 4 8; do
  PT_PIPE_DEPTH=$d timeout -k 10 300 python -u tools/tune.py --config c2 --frames 100 --rounds 3 > "gpurun_out/r_c2_d$d.log" 2>&1; rc=$?
  echo "c2 depth $d: $(tail -1 gpurun_out/r_c2_d$d.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
done
