#!/usr/bin/env python3
"""DRAM-side bytes per frame of a config's frame kernel for each build of tools/gpu_attr.sh.

    python tools/attr.py c4 base nostore envsmall

dram = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (KiB units, gfx950's FETCH_SIZE halving; see
tools/roofline.py), of the frame kernel's last dispatch (one of the bench's timed launches) divided by the frames it
renders (the bench line's frames_per_launch)."""
import csv
import glob
import json
import sys


def kernel_kb(path, counter):
    rows = [r for r in csv.DictReader(open(glob.glob(path + "/**/*counter_collection.csv", recursive=True)[0]))
            if r["Counter_Name"] == counter and ("renderKernel" in r["Kernel_Name"] or "regenKernel" in r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    per = {}
    for r in rows:
        per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return list(per.values())[-1]  # the timed frames' last launch (frames_per_launch frames)


def frames_per_launch(log):
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)["config"].get("frames_per_launch") or 1
    return 1


def main():
    cfg, variants = sys.argv[1], sys.argv[2:]
    for v in variants:
        d = f"gpurun_out/attr_{cfg}_{v}"
        f = frames_per_launch(d + "/fetch.log")
        fetch, write = kernel_kb(d + "/fetch", "FETCH_SIZE"), kernel_kb(d + "/write", "WRITE_SIZE")
        print(f"{cfg} {v:10s} frames/launch {f:2d}  read {2 * fetch * 1024 / f / 1e6:7.1f} MB  "
              f"write {write * 1024 / f / 1e6:7.1f} MB  dram {(2 * fetch + write) * 1024 / f / 1e6:7.1f} MB per frame")


if __name__ == "__main__":
    main()
