#!/bin/bash
# experiments: grid oversubscription for frames in flight (PT_GRID_PCT) at N = 1 / 8 shares,
# and the regen kernel's dynamic ray fetch variants (PT_REGEN_YIELD) on c5 (digest + timing)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; O=$R/gpurun_out/exp2; mkdir -p $O; cd $R
for v in ${VARIANTS:-y8 y16 y32 y48 y16w3}; do
  timeout -k 10 200 python tools/variant_digest.py base $v --config c5 --frames 2 >> $O/digest.jsonl 2>>$O/err.log; rc=$?
  echo digest $v rc=$rc; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 500 python tools/tune.py --variants base ${VARIANTS:-y8 y16 y32 y48 y16w3} --config c5 --frames 30 --warmup 10 --rounds 2 > $O/tune_c5.jsonl 2>>$O/err.log; rc=$?
echo tune rc=$rc; [ $rc -eq 0 ] || exit $rc
for pct in ${PCTS:-150 200 300 800}; do for c in c2 c4; do
  echo "pct=$pct" >> $O/pct.jsonl
  PT_GRID_PCT=$pct timeout -k 10 200 python tools/shard_time.py $c 1 8 >> $O/pct.jsonl 2>>$O/err.log; rc=$?; echo pct=$pct $c rc=$rc; [ $rc -eq 0 ] || exit $rc
done; done
cat $O/digest.jsonl $O/pct.jsonl; tail -1 $O/tune_c5.jsonl
