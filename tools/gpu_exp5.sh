#!/bin/bash
# the large-scene regen path (4-wide walk, dynamic ray fetch, camera-ray pass) on the small
# scenes (PT_REGEN_WIDE=1) vs the megakernel: digests and wall ms/frame; c5's 3-wave regen variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out/exp5; mkdir -p $O; cd $R
for c in c4 c2 c3; do
  for rw in 0 1; do
    PT_REGEN_WIDE=$rw timeout -k 10 200 python tools/variant_digest.py base base --config $c --frames 3 > $O/digest_${c}_$rw.jsonl 2>>$O/err.log; rc=$?
    echo digest $c regen_wide=$rw rc=$rc; head -1 $O/digest_${c}_$rw.jsonl; [ $rc -le 1 ] || exit $rc
  done
done
for c in c4 c2 c3; do for rw in 0 1 0 1; do
  PT_REGEN_WIDE=$rw timeout -k 10 200 python tools/tune.py --config $c --frames 60 --warmup 100 --rounds 1 > $O/t.jsonl 2>>$O/err.log; rc=$?
  echo "regen_wide=$rw $(tail -1 $O/t.jsonl)"; [ $rc -eq 0 ] || exit $rc
done; done
if [ -f opengl_ray_tracing_amd/_variants/libpt_w3.so ]; then
  timeout -k 10 400 python tools/tune.py --variants base w3 --config c5 --frames 30 --warmup 100 --rounds 2 > $O/tune_c5.jsonl 2>>$O/err.log; rc=$?
  echo c5 rc=$rc; tail -1 $O/tune_c5.jsonl; [ $rc -eq 0 ] || exit $rc
fi
