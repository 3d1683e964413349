#!/bin/bash
# GPU tests, then frames-in-flight work sharing on/off (PT_SHARE_WORK) for one rank's share of
# the screen-tile split (tools/shard_time.py), then the regen kernel's yield sweep on c5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out/exp3; mkdir -p $O; cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo pytest=$rc; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for sw in ${SHARES:-1 0 1}; do for c in c2 c4; do
  echo "share=$sw" >> $O/share.jsonl
  PT_SHARE_WORK=${sw%%:*} PT_SHARE_AHEAD=${sw#*:} timeout -k 10 240 python tools/shard_time.py $c 1 2 4 8 >> $O/share.jsonl 2>>$O/err.log; rc=$?
  echo share=$sw $c rc=$rc; [ $rc -eq 0 ] || exit $rc
done; done
cat $O/share.jsonl
if [ -n "$VARIANTS" ]; then
  timeout -k 10 500 python tools/tune.py --variants base $VARIANTS --config c5 --frames 30 --warmup 10 --rounds 2 > $O/tune_c5.jsonl 2>>$O/err.log; rc=$?
  echo tune rc=$rc; tail -1 $O/tune_c5.jsonl; [ $rc -eq 0 ] || exit $rc
fi
