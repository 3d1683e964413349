#!/usr/bin/env python3
"""Copy the judged evidence of tools/gpu_evidence.sh from gpurun_out/ into profiles/<round>/.

    python tools/collect_evidence.py r1 c2 c4 c5

profiles/<round>/<cfg>/kernel_stats.csv  rocprofv3 --kernel-trace --stats summary
profiles/<round>/<cfg>/{fetch,write}_size.csv  FETCH_SIZE / WRITE_SIZE rows of the frame kernels
profiles/<round>/bench_<cfg>.json  the bench line, profiles/<round>/traffic.json  per-launch HBM bytes
"""
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"


def main():
    tag, cfgs = sys.argv[1], sys.argv[2:] or ["c2", "c4", "c5"]
    dst = ROOT / "profiles" / tag
    dst.mkdir(parents=True, exist_ok=True)
    for c in cfgs:
        d = dst / c
        d.mkdir(exist_ok=True)
        prof = OUT / f"prof_{tag}_{c}"
        shutil.copy(prof / "trace" / "run_kernel_stats.csv", d / "kernel_stats.csv")
        for name in ("fetch", "write"):
            lines = (prof / name / "run_counter_collection.csv").read_text().splitlines()
            keep = [lines[0]] + [ln for ln in lines[1:] if "renderKernel" in ln]
            (d / f"{name}_size.csv").write_text("\n".join(keep) + "\n")
        shutil.copy(OUT / f"bench_{c}.json", dst / f"bench_{c}.json")
    shutil.copy(OUT / "traffic.json", dst / "traffic.json")
    print("evidence ->", dst)


if __name__ == "__main__":
    main()
