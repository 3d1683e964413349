#!/usr/bin/env python3
"""Roofline evidence from the rocprofv3 runs of tools/gpu_profile.sh.

    python tools/roofline.py <tag> <cfg> [<cfg> ...]

Reads gpurun_out/prof_<tag>_<cfg>/ and writes, under profiles/<tag>/:
  <cfg>/kernel_stats.csv       rocprofv3 --kernel-trace --stats summary of the bench command
  <cfg>/timed_dispatches.json  the bench kernel's dispatches of bench.py's timed region
  <cfg>/counters.csv           every counter row of the bench kernel's timed dispatches
  bench_<cfg>.json             the profiled run's bench line
  counters.json                {cfg: per-launch counter averages + the derived roofline work}
bench.py reads counters.json (--counters) and divides each resource's per-launch
work by its own live kernel time.

The bench kernel is the culling frame kernel renderKernel<I, true, false[, W]>
(or, for large Disney/MIS scenes, the path-regeneration kernel regenKernel<I, true[, W]>).
bench.py renders PROBE_FRAMES policy-probe frames, then W warmup and K timed
frames of it, so its timed dispatches are numbers [PROBE+W, PROBE+W+K) in
dispatch order (the fetch-counting kernel, renderKernel<I, false, true>, and
the PSNR check's basicKernel are other kernels).

Derived per-launch work (MI355X_MICROARCH.md):
  valu_insts = SQ_INSTS_VALU (wave64 instructions; peak issue 1024 SIMDs x 2.4 GHz / 2 cycles)
  dram_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (KiB units; gfx950 FETCH_SIZE halving)
  l2_hit     = TCC_HIT / (TCC_HIT + TCC_MISS);  clock_ghz = GRBM_GUI_ACTIVE / 8 / dispatch time, per sq-pass dispatch
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
PROBE = 90  # bench.py PROBE_FRAMES: policy-probe frames ahead of the warmup and timed frames
TRACE_RUN = (5, 30)    # tools/gpu_profile.sh: --warmup 5 --steps 30 under --kernel-trace
COUNTER_RUN = (2, 10)  # --warmup 2 --steps 10 under each --pmc pass
BENCH_KERNEL = re.compile(r"renderKernel<\d+, true, false(, \d+)?>|regenKernel<\d+, true(, \d+)?(, (true|false))?>")


def one(pattern: str) -> Path:
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return Path(hits[0])


def timed(rows, run):
    w, k = run
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    return rows[PROBE + w:PROBE + w + k], len(rows)


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
        trace = [r for r in csv.DictReader(open(one(f"{prof}/trace/**/run_kernel_trace.csv")))
                 if BENCH_KERNEL.search(r["Kernel_Name"])]
        sel, total = timed(trace, TRACE_RUN)
        ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
        kernel_ms = sum(ms) / len(ms)
        (d / "timed_dispatches.json").write_text(json.dumps({
            "kernel": sel[-1]["Kernel_Name"], "dispatches": total, "timed_dispatches": len(sel),
            "selection": f"dispatches [{PROBE}+{TRACE_RUN[0]}, +{TRACE_RUN[1]}) of the bench kernel",
            "timed_avg_ms": round(kernel_ms, 4), "timed_ms": [round(x, 4) for x in ms],
            "vgpr": sel[-1].get("VGPR_Count"), "scratch": sel[-1].get("Scratch_Size")}, indent=1) + "\n")
        line = (prof / "bench_line.json").read_text().strip().splitlines()
        line = [ln for ln in line if ln.startswith("{")]
        if line:
            (dst / f"bench_{c}.json").write_text(line[-1] + "\n")

        vals = defaultdict(list)
        rows_out = []
        header = None
        for name in ("fetch", "write", "sq", "mem"):
            f = one(f"{prof}/{name}/**/run_counter_collection.csv")
            rows = list(csv.DictReader(open(f)))
            header = header or list(rows[0].keys())
            bench = [r for r in rows if BENCH_KERNEL.search(r["Kernel_Name"])]
            by_disp = defaultdict(list)
            for r in bench:
                by_disp[r["Dispatch_Id"]].append(r)
            disp = sorted(by_disp, key=int)
            w, k = COUNTER_RUN
            keep = disp[PROBE + w:PROBE + w + k]
            for di in keep:
                for r in by_disp[di]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                    rows_out.append({"pass": name, **r})
                r0 = by_disp[di][0]
                if name == "sq" and r0.get("End_Timestamp"):  # the counter pass's own dispatch duration
                    dms = (int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])) / 1e6
                    vals["_counter_dispatch_ms"].append(dms)
                    # the clock of this dispatch: its own GRBM_GUI_ACTIVE (8 XCDs) over its own duration
                    # (GRBM_GUI_ACTIVE is also sampled in the mem pass, whose dispatches last differently)
                    gg = [float(r["Counter_Value"]) for r in by_disp[di] if r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
                    if gg and dms > 0:
                        vals["_clock_ghz"].append(gg[0] / 8 / (dms * 1e-3) / 1e9)
        with open(d / "counters.csv", "w", newline="") as fh:
            wr = csv.DictWriter(fh, fieldnames=["pass"] + header)
            wr.writeheader()
            wr.writerows(rows_out)
        m = {k: sum(v) / len(v) for k, v in vals.items()}
        g = lambda k: m.get(k, float("nan"))  # noqa: E731
        cms = m.pop("_counter_dispatch_ms", float("nan"))
        vals.pop("_counter_dispatch_ms", None)
        clock = m.pop("_clock_ghz", float("nan"))
        vals.pop("_clock_ghz", None)
        # the kernel with nothing overlapping it: the serial-frames trace (PT_FLAG_SERIAL_FRAMES)
        serial_ms = None
        sp = sorted(glob.glob(f"{prof}/serial/**/run_kernel_trace.csv", recursive=True))
        if sp:
            st = [r for r in csv.DictReader(open(sp[0])) if BENCH_KERNEL.search(r["Kernel_Name"])]
            ssel, _ = timed(st, TRACE_RUN)
            sms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ssel]
            serial_ms = round(sum(sms) / len(sms), 4)
            shutil.copy(one(f"{prof}/serial/**/run_kernel_stats.csv"), d / "kernel_stats_serial.csv")
        ent = {
            "kernel": sel[-1]["Kernel_Name"], "kernel_ms": round(kernel_ms, 4),
            "valu_insts": round(g("SQ_INSTS_VALU")),
            "dram_bytes": round((2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024),
            "l2_hit": round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 4),
            "valu_lane_util": round(g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU")), 4),
            # per dispatch of the sq pass: GRBM_GUI_ACTIVE summed over the 8 XCDs over that dispatch's
            # own (serialised) duration -- the interval its counters describe -- averaged
            "counter_dispatch_ms": round(cms, 4),
            "clock_ghz_profiled": round(clock, 3),
            "serial_kernel_ms": serial_ms,
            "counters_per_launch": {k: round(v, 1) for k, v in sorted(m.items())},
            "samples": {k: len(v) for k, v in sorted(vals.items())},
            "derivation": "valu_insts = SQ_INSTS_VALU; dram_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024; "
                          "per launch, averaged over the bench kernel's timed dispatches of each pass",
        }
        summary[c] = ent
        print(c, json.dumps({k: ent[k] for k in ("kernel_ms", "serial_kernel_ms", "counter_dispatch_ms", "valu_insts",
                                                  "dram_bytes", "l2_hit", "valu_lane_util", "clock_ghz_profiled")}))
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
    cand = {
        "valu": {"achieved": round(ent["valu_insts"] / t / 1e9, 2), "peak": VALU_PEAK_GINST,
                 "unit": "G VALU wave-instructions/s"},
        "hbm": {"achieved": round(ent["dram_bytes"] / t / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s"},
    }
    for v in cand.values():
        v["frac"] = round(v["achieved"] / v["peak"], 4)
    bound = max(cand, key=lambda k: cand[k]["frac"])
    rf.update({"bound": bound, **{k: cand[bound][k] for k in ("achieved", "peak", "unit", "frac")},
               "traffic": ent["dram_bytes"], "candidates": cand,
               "counters": {"source": f"profiles/{path.parent.name}/counters.json", "valu_insts_per_launch": ent["valu_insts"],
                            "dram_bytes_per_launch": ent["dram_bytes"], "l2_hit": ent["l2_hit"],
                            "profiled_kernel_ms": ent["kernel_ms"]},
               "restated_from_counters_of_this_run": True})
    line["roofline"] = rf
    path.write_text(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
