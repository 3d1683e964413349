#!/usr/bin/env python3
"""Roofline evidence from the rocprofv3 runs of tools/gpu_profile.sh, over every kernel of a frame.

    python tools/roofline.py <tag> <cfg> [<cfg> ...]

Reads gpurun_out/prof_<tag>_<cfg>/ and writes, under profiles/<tag>/:
  <cfg>/kernel_stats.csv        rocprofv3 --kernel-trace --stats summary of the bench command
  <cfg>/kernel_stats_serial.csv the same with frames issued serially (PT_FLAG_SERIAL_FRAMES)
  <cfg>/timed_dispatches.json   each frame kernel's dispatches of bench.py's timed frames
  <cfg>/counters.csv            every counter row of those dispatches
  bench_<cfg>.json              the profiled run's bench line
  counters.json                 {cfg: per-kernel and per-frame counter work, time bases}

A frame (bench.py step at N = 1) runs these kernels, each once (FRAME_KERNELS): the camera-ray
pass primaryKernel (the regen path), the frame kernel (renderKernel<I, true, false[, W]> or
regenKernel<I, true[, W, true]>), the tile reorder reorderKernel (megakernel frames in
longest-first order) and the running-mean update mixKernel. The profiled bench runs end with its
timed frames (--no-reset --no-serial --no-psnr), so each kernel's last K dispatches are the timed
frames' (K = the run's --steps).

Per kernel (averaged over its timed dispatches of each pass, divided by the frames a dispatch
renders: the bench's frames_per_launch) and summed per frame:
  valu_insts = SQ_INSTS_VALU (wave64 instructions; peak issue 1024 SIMDs x 2.4 GHz / 2 cycles)
  dram_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (KiB units; gfx950 FETCH_SIZE halving)
  l2_hit     = TCC_HIT / (TCC_HIT + TCC_MISS)
Time bases: the pipelined trace's wall time per frame is bench.py's (ms_per_step); the summed
serial-trace durations of the frame's kernels (frames issued one after another, accumulating in
place: no mixKernel) are its kernel basis -- divided into the work of the same kernels.
bench.py reads counters.json (--counters): frame.valu_insts / frame.dram_bytes over the wall time,
frame_serial.* over the serial kernel time.
"""
import csv
import glob
import json
import re
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"
# tools/gpu_profile.sh: --steps 32 under --kernel-trace (pipelined and serial), --steps 16 under each
# --pmc pass -- multiples of every automatic frames-per-launch (1, 2, 4, 8, 16), so the last
# steps / F dispatches are exactly the timed frames (round 4's first c4 profile at 30 / 10 with F = 4
# averaged a 2-frame launch in and under-counted its frames by a quarter)
TRACE_STEPS = 96  # divisible by every frames-per-launch the bench uses (12 for c2, 32 for c4, 2 for c5)
COUNTER_STEPS = 96
FRAME_KERNELS = {
    "primary": re.compile(r"primaryKernel"),
    "frame": re.compile(r"renderKernel<\d+, true, false(, \d+)?>|regenKernel<\d+, true[^>]*>"),
    "reorder": re.compile(r"reorderKernel"),
    "mix": re.compile(r"mixKernel"),
}


def one(pattern: str) -> Path:
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return Path(hits[0])


def kind_of(name):
    for k, rx in FRAME_KERNELS.items():
        if rx.search(name):
            return k
    return None


def last_dispatches(rows, k):
    """{kind: the last k dispatches of that frame kernel, in dispatch order}"""
    by = defaultdict(list)
    for r in rows:
        kd = kind_of(r["Kernel_Name"])
        if kd:
            by[kd].append(r)
    return {kd: sorted(v, key=lambda r: int(r["Dispatch_Id"]))[-k:] for kd, v in by.items()}


def dur_ms(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6


def main():
    tag, cfgs = sys.argv[1], sys.argv[2:] or ["c2", "c4", "c5"]
    dst = ROOT / "profiles" / tag
    dst.mkdir(parents=True, exist_ok=True)
    cpath = dst / "counters.json"
    summary = json.loads(cpath.read_text()) if cpath.exists() else {}
    for c in cfgs:
        prof = OUT / f"prof_{tag}_{c}"
        d = dst / c
        d.mkdir(exist_ok=True)
        shutil.copy(one(f"{prof}/trace/**/run_kernel_stats.csv"), d / "kernel_stats.csv")
        # frames per launch of the profiled bench (pt_render_frames_async batches): each frame kernel's
        # dispatch covers F frames, so the timed frames are the last steps / F dispatches and a
        # dispatch's work is F frames' work
        bl = [ln for ln in (prof / "bench_line.json").read_text().splitlines() if ln.startswith("{")]
        F = int(json.loads(bl[-1])["config"].get("frames_per_launch") or 1) if bl else 1
        trace = list(csv.DictReader(open(one(f"{prof}/trace/**/run_kernel_trace.csv"))))
        sel = last_dispatches(trace, max(1, TRACE_STEPS // F))
        serial = {}
        sp = sorted(glob.glob(f"{prof}/serial/**/run_kernel_trace.csv", recursive=True))
        if sp:
            serial = last_dispatches(list(csv.DictReader(open(sp[0]))), TRACE_STEPS)
            shutil.copy(one(f"{prof}/serial/**/run_kernel_stats.csv"), d / "kernel_stats_serial.csv")
        disp = {}
        for kd, rows in sel.items():
            ms = [dur_ms(r) for r in rows]
            disp[kd] = {"kernel": rows[-1]["Kernel_Name"], "timed_dispatches": len(rows), "frames_per_dispatch": F,
                        "avg_ms_pipelined": round(sum(ms) / len(ms), 4), "min_ms_pipelined": round(min(ms), 4),
                        "vgpr": rows[-1].get("VGPR_Count"), "scratch": rows[-1].get("Scratch_Size")}
            if kd in serial:
                sms = [dur_ms(r) for r in serial[kd]]
                disp[kd]["avg_ms_serial"] = round(sum(sms) / len(sms), 4)
        (d / "timed_dispatches.json").write_text(json.dumps({
            "selection": f"the last {TRACE_STEPS} dispatches of each frame kernel (the bench's timed frames)",
            "kernels": disp}, indent=1) + "\n")
        line = (prof / "bench_line.json").read_text().strip().splitlines()
        line = [ln for ln in line if ln.startswith("{")]
        if line:
            (dst / f"bench_{c}.json").write_text(line[-1] + "\n")

        vals = {kd: defaultdict(list) for kd in FRAME_KERNELS}
        rows_out = []
        header = None
        for name in ("fetch", "write", "sq", "mem"):
            rows = list(csv.DictReader(open(one(f"{prof}/{name}/**/run_counter_collection.csv"))))
            header = header or list(rows[0].keys())
            by_disp = defaultdict(list)
            for r in rows:
                if kind_of(r["Kernel_Name"]):
                    by_disp[r["Dispatch_Id"]].append(r)
            per_kind = defaultdict(list)
            for di in sorted(by_disp, key=int):
                per_kind[kind_of(by_disp[di][0]["Kernel_Name"])].append(di)
            for kd, dis in per_kind.items():
                for di in dis[-max(1, COUNTER_STEPS // F):]:
                    for r in by_disp[di]:
                        vals[kd][r["Counter_Name"]].append(float(r["Counter_Value"]))
                        rows_out.append({"pass": name, **r})
                    r0 = by_disp[di][0]
                    if name == "sq" and r0.get("End_Timestamp"):  # the dispatch's own (serialised) duration
                        vals[kd]["_dispatch_ms"].append(dur_ms(r0))
        with open(d / "counters.csv", "w", newline="") as fh:
            wr = csv.DictWriter(fh, fieldnames=["pass"] + header)
            wr.writeheader()
            wr.writerows(rows_out)
        kernels = {}
        for kd, v in vals.items():
            if not v:
                continue
            # per frame: a dispatch's counters over the F frames it rendered (time keys stay per dispatch)
            m = {k: sum(x) / len(x) / (1 if k.startswith("_") else F) for k, x in v.items()}
            g = lambda k: m.get(k, float("nan"))  # noqa: E731
            kernels[kd] = {
                "kernel": disp.get(kd, {}).get("kernel"),
                "valu_insts": round(g("SQ_INSTS_VALU")),
                "dram_bytes": round((2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024),
                "l2_hit": round(g("TCC_HIT_sum") / max(g("TCC_HIT_sum") + g("TCC_MISS_sum"), 1.0), 4),
                "valu_lane_util": round(g("SQ_THREAD_CYCLES_VALU") / max(64 * g("SQ_ACTIVE_INST_VALU"), 1.0), 4),
                "counter_dispatch_ms": round(g("_dispatch_ms") / F, 4),  # per frame
                "avg_ms_serial": disp.get(kd, {}).get("avg_ms_serial"),
                "avg_ms_pipelined": disp.get(kd, {}).get("avg_ms_pipelined"),
                "counters_per_launch": {k: round(x, 1) for k, x in sorted(m.items()) if not k.startswith("_")},
            }

        def frame_sum(kinds):
            ks = [kernels[k] for k in kinds if k in kernels]
            return {"kernels": [k for k in kinds if k in kernels],
                    "valu_insts": sum(k["valu_insts"] for k in ks), "dram_bytes": sum(k["dram_bytes"] for k in ks),
                    "counter_dispatch_ms": round(sum(k["counter_dispatch_ms"] for k in ks), 4)}
        frame = frame_sum(list(FRAME_KERNELS))
        fserial = frame_sum([k for k in FRAME_KERNELS if k != "mix"])
        ser = [kernels[k]["avg_ms_serial"] for k in fserial["kernels"] if kernels[k].get("avg_ms_serial")]
        fserial["serial_kernel_ms"] = round(sum(ser), 4) if ser else None
        fk = kernels.get("frame", {})
        ent = {
            # the frame kernel alone (as rounds 1-3 reported it) ...
            "kernel": fk.get("kernel"), "valu_insts": fk.get("valu_insts"), "dram_bytes": fk.get("dram_bytes"),
            "l2_hit": fk.get("l2_hit"), "valu_lane_util": fk.get("valu_lane_util"),
            "kernel_ms": disp.get("frame", {}).get("avg_ms_pipelined"),
            "serial_kernel_ms": disp.get("frame", {}).get("avg_ms_serial"),
            # ... and every kernel of a frame
            "kernels": kernels,
            "frames_per_launch": F,
            "frame": frame,            # all frame kernels: work over bench.py's wall ms per frame
            "frame_serial": fserial,   # without mixKernel: work over the serial frames' kernel time
            "derivation": "per kernel: valu_insts = SQ_INSTS_VALU; dram_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024, "
                          f"averaged over its last {COUNTER_STEPS} dispatches (the timed frames) of each --pmc pass; "
                          "frame = the sum over the frame's kernels (each runs once per frame)",
        }
        summary[c] = ent
        print(c, json.dumps({"frame": frame, "frame_serial": fserial,
                             "per_kernel": {k: (v["valu_insts"], v["dram_bytes"], v["counter_dispatch_ms"])
                                            for k, v in kernels.items()}}))
        restate(dst / f"bench_{c}.json", ent)
    cpath.write_text(json.dumps(summary, indent=1) + "\n")


VALU_PEAK_GINST = 1024 * 2.4 / 2  # bench.py: 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction
HBM_PEAK_GBS = 8000.0


def restate(path: Path, ent: dict):
    """The profiled bench line read the counters committed before this run; restate its
    roofline with the counters just measured (same formulas as bench.py make_roofline), so
    every committed frac is the committed per-launch work over the line's own time basis."""
    if not path.exists():
        return
    line = json.loads(path.read_text())
    rf = line.get("roofline") or {}
    t = line["ms_per_step"] if rf.get("time_basis", "").startswith("wall") else rf.get("launch_ms", line["ms_per_step"])
    t *= 1e-3
    work = ent["frame"] if rf.get("time_basis", "").startswith("wall") else ent["frame_serial"]
    cand = {
        "valu": {"achieved": round(work["valu_insts"] / t / 1e9, 2), "peak": VALU_PEAK_GINST,
                 "unit": "G VALU wave-instructions/s"},
        "hbm": {"achieved": round(work["dram_bytes"] / t / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s"},
    }
    for v in cand.values():
        v["frac"] = round(v["achieved"] / v["peak"], 4)
    bound = max(cand, key=lambda k: cand[k]["frac"])
    rf.update({"bound": bound, **{k: cand[bound][k] for k in ("achieved", "peak", "unit", "frac")},
               "traffic": work["dram_bytes"], "candidates": cand,
               "counters": {"source": f"profiles/{path.parent.name}/counters.json", "kernels": work["kernels"],
                            "valu_insts_per_frame": work["valu_insts"], "dram_bytes_per_frame": work["dram_bytes"],
                            "l2_hit": ent["l2_hit"], "profiled_kernel_ms": ent["kernel_ms"]},
               "restated_from_counters_of_this_run": True})
    line["roofline"] = rf
    path.write_text(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
