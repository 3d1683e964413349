#!/usr/bin/env python3
"""Copy the judged evidence of tools/gpu_evidence.sh from gpurun_out/ into profiles/<round>/.

    python tools/collect_evidence.py r1 c2 c4 c5

profiles/<round>/<cfg>/kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
profiles/<round>/<cfg>/{fetch,write}_size.csv  FETCH_SIZE / WRITE_SIZE rows of the frame kernels
profiles/<round>/bench_<cfg>.json  the bench line, profiles/<round>/traffic.json  per-launch HBM bytes
profiles/<round>/<cfg>/timed_dispatches.json  the profiled run's bench-kernel dispatches: the last
    STEPS (its timed region, the same one bench.py's HIP events average) and all of them (with the
    runtime's probe frames and the warmup, which kernel_stats.csv averages)
"""
import csv
import json
import re
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"
STEPS = 30  # tools/gpu_profile.sh: bench.py --steps 30 under rocprofv3 --kernel-trace
BENCH_KERNEL = re.compile(r"renderKernel<\d+, true, false(, \d+)?>")


def timed_dispatches(trace_csv: Path) -> dict:
    rows = [r for r in csv.DictReader(open(trace_csv)) if BENCH_KERNEL.search(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    last = ms[-STEPS:]
    return {"kernel": rows[-1]["Kernel_Name"] if rows else None, "dispatches": len(ms),
            "timed_dispatches": len(last), "timed_avg_ms": round(sum(last) / max(len(last), 1), 4),
            "all_avg_ms": round(sum(ms) / max(len(ms), 1), 4), "timed_ms": [round(x, 4) for x in last]}


def main():
    tag, cfgs = sys.argv[1], sys.argv[2:] or ["c2", "c4", "c5"]
    dst = ROOT / "profiles" / tag
    dst.mkdir(parents=True, exist_ok=True)
    for c in cfgs:
        d = dst / c
        d.mkdir(exist_ok=True)
        prof = OUT / f"prof_{tag}_{c}"
        shutil.copy(prof / "trace" / "run_kernel_stats.csv", d / "kernel_stats.csv")
        (d / "timed_dispatches.json").write_text(json.dumps(timed_dispatches(prof / "trace" / "run_kernel_trace.csv"),
                                                            indent=1) + "\n")
        for name in ("fetch", "write"):
            lines = (prof / name / "run_counter_collection.csv").read_text().splitlines()
            keep = [lines[0]] + [ln for ln in lines[1:] if "renderKernel" in ln]
            (d / f"{name}_size.csv").write_text("\n".join(keep) + "\n")
        shutil.copy(OUT / f"bench_{c}.json", dst / f"bench_{c}.json")
    shutil.copy(OUT / "traffic.json", dst / "traffic.json")
    print("evidence ->", dst)


if __name__ == "__main__":
    main()
