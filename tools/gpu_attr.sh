#!/bin/bash
# DRAM-side traffic attribution of a config's frame kernel: the FETCH_SIZE and WRITE_SIZE passes of
# tools/gpu_profile.sh over the bench's pipelined frames, once per tuning build (diagnostics builds
# such as PT_DIAG_NO_STORE / PT_DIAG_ENV_SMALL remove one buffer's traffic; "base" = libpt.so).
#   bash tools/gpu_attr.sh c4 base nostore envsmall   -> gpurun_out/attr_<cfg>_<variant>/; tools/attr.py
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CFG=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  OUT="$REPO/gpurun_out/attr_${CFG}_$v"; mkdir -p "$OUT"
  for p in "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
    name="${p%%:*}"; ctr="${p#*:}"
    if [ "$v" = base ]; then unset PT_VARIANT; else export PT_VARIANT=$v; fi
    timeout -s KILL 300 rocprofv3 --pmc $ctr -f csv -d "$OUT/$name" -o run -- \
      python3 "$REPO/bench.py" --config "$CFG" --steps 16 --warmup 2 --no-cpu-baseline --no-psnr --no-reset --no-serial \
      > "$OUT/$name.log" 2>&1; rc=$?
    echo "$v $name=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
