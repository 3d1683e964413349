#!/bin/bash
# A/B of environment switches on one rank's share (tools/shard_time.py): CFG FRAMES "N..." then
# quoted VAR=VALUE lists, "" = the default.   bash tools/ab_c4_policy.sh c4 20 "1 8" "" "PT_ORDER=1"
set -o pipefail
CFG=$1; F=$2; NS=$3; shift 3
for v in "$@"; do
  env $v PT_SHARD_FRAMES=$F timeout -k 10 200 python tools/shard_time.py $CFG $NS > gpurun_out/ab_env.log 2>&1 || exit $?
  echo "[$v] $(grep -o '"rank0_ms_per_frame": [0-9.]*' gpurun_out/ab_env.log | cut -d' ' -f2 | tr '\n' ' ')"
done
