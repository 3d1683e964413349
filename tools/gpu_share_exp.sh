set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/share; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/tools/shard_time.py c2 8 > $O/trace.out 2>&1; rc=$?; echo trace=$rc; [ $rc -eq 0 ] || exit $rc
cd $R
for pct in 100 90 75; do for c in c2 c4; do
  echo "pct=$pct" >> $O/pct.jsonl
  PT_GRID_PCT=$pct timeout -k 10 200 python tools/shard_time.py $c 1 8 >> $O/pct.jsonl 2>>$O/err.log; rc=$?; echo pct=$pct $c rc=$rc; [ $rc -eq 0 ] || exit $rc
done; done
for d in 12 16; do for c in c2 c4; do
  echo "depth=$d" >> $O/pct.jsonl
  GPU_MAX_HW_QUEUES=20 PT_PIPE_DEPTH=$d timeout -k 10 200 python tools/shard_time.py $c 1 8 >> $O/pct.jsonl 2>>$O/err.log; rc=$?; echo depth=$d $c rc=$rc; [ $rc -eq 0 ] || exit $rc
done; done
cat $O/pct.jsonl
