#!/bin/bash
# Hardware-queue assignment of HIP streams (tools/probe/queue_map.hip) under the environment's
# GPU_MAX_HW_QUEUES: prints, per spin kernel (grid size = stream index + 1), its Queue_Id.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
OUT="$REPO/gpurun_out/qmap_${1:-6}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --kernel-trace -f csv -d "$OUT" -o run -- "$REPO/tools/probe/queue_map" "${1:-6}" > "$OUT/log.txt" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "spin" in r["Kernel_Name"]]
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    print("stream", int(r["Grid_Size"]) // 64 - 1, "queue", r["Queue_Id"], "start", r["Start_Timestamp"], "end", r["End_Timestamp"])
PY
