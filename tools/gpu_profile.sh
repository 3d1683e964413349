#!/bin/bash
# rocprofv3 evidence for the bench kernel of config $2 (tag $1): kernel trace +
# stats of the bench command, then the counter groups the roofline needs, each
# in its own rocprofv3 pass (--pmc with kernel dispatch records only; FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950). Output: gpurun_out/prof_<tag>_<cfg>/.
# Summarise with tools/roofline.py.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2}"
CFG="${2:-c2}"
OUT="$REPO/gpurun_out/prof_${TAG}_${CFG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# the bench's own flow: 14 probe frames, W warmup, K timed frames (tools/roofline.py selects those)
BENCH=(python3 "$REPO/bench.py" --config "$CFG" --steps 96 --warmup 5 --no-cpu-baseline --no-psnr --no-reset --no-serial --no-per-call)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- "${BENCH[@]}" > "$OUT/bench_line.json" 2> "$OUT/trace.log"; rc=$?
echo "trace=$rc"; [ $rc -eq 0 ] || exit $rc
# the same flow with frames issued serially (PT_FLAG_SERIAL_FRAMES = 0x80): the kernel's own duration
SERIAL=(python3 "$REPO/bench.py" --config "$CFG" --steps 96 --warmup 5 --no-cpu-baseline --no-psnr --no-reset --no-serial --no-per-call --flags 128)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/serial" -o run -- "${SERIAL[@]}" > "$OUT/serial_line.json" 2> "$OUT/serial.log"; rc=$?
echo "serial=$rc"; [ $rc -eq 0 ] || exit $rc
# counters over the bench's own (pipelined) frames: a --pmc pass serialises the dispatches, so each
# frame kernel's counters -- camera-ray pass, frame kernel, tile reorder, running-mean update --
# cover its own dispatch (tools/roofline.py sums them per frame)
BENCHC=(python3 "$REPO/bench.py" --config "$CFG" --steps 96 --warmup 2 --no-cpu-baseline --no-psnr --no-reset --no-serial --no-per-call)
PASSES=(
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
  "sq:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
  "mem:TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
)
for p in "${PASSES[@]}"; do
  name="${p%%:*}"; ctr="${p#*:}"
  timeout -s KILL 300 rocprofv3 --pmc $ctr -f csv -d "$OUT/$name" -o run -- "${BENCHC[@]}" > "$OUT/$name.log" 2>&1; rc=$?
  echo "pass $name=$rc"; [ $rc -eq 0 ] || exit $rc
done
