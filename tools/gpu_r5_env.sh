#!/bin/bash
# Round-5 A/B: compact env texels (PT_ENV_COMPACT=1, default) against float texels, bench lines of
# c2/c3/c4/c5 at the box's hardware queues, then DRAM-side bytes of c4's frame kernel both ways.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/env
for rep in 1 2; do
  for cfg in c2 c3 c4; do
    for ce in 1 0; do
      PT_ENV_COMPACT=$ce timeout -k 10 300 python bench.py --config $cfg --steps 40 --warmup 5 --no-cpu-baseline --no-psnr --no-serial --no-reset > gpurun_out/env/${cfg}_$ce.json 2>/dev/null || exit 1
      echo "$cfg compact=$ce rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/env/${cfg}_$ce.json)"
    done
  done
done
for ce in 1 0; do
  PT_ENV_COMPACT=$ce timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-psnr --no-serial --no-reset > gpurun_out/env/c5_$ce.json 2>/dev/null || exit 1
  echo "c5 compact=$ce $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/env/c5_$ce.json)"
done
cd /tmp && export TMPDIR=/tmp
for ce in 1 0; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PT_ENV_COMPACT=$ce timeout -s KILL 120 rocprofv3 --pmc $ctr -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/env/pmc_${ce}_$ctr" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --config c4 --steps 16 --warmup 2 --no-cpu-baseline --no-psnr --no-reset --no-serial > /dev/null 2>&1 || exit 1
  done
done
echo pmc done
