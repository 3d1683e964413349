#!/usr/bin/env python3
"""What the reference's caller gets per display(): the wall time of one synchronous
pt_render_frame call (median of 100 calls after 10 warm-up calls), per config.

The reference draws one frame per display() (OpenglRayTracing/main.cpp:558-603, IS main.cpp:659-709);
INTEGRATION.md binds one pt_render_frame per display(). Each call here renders frame k of one
camera and returns when its running-mean update is complete (the call's own synchronisation).

    python tools/per_call.py [c2 c4 ...] [--calls 100] [--warmup 10]

Prints one JSON line per config: median / p10 / p90 wall ms per call and the Mrays/s of the
median call (rays per frame from the renderer's counters over the timed calls).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import opengl_ray_tracing_amd  # noqa: E402,F401  (hardware-queue policy before HIP initialises)
from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes  # noqa: E402

PROBE_FRAMES = 90  # bench.py's: the renderer's policy probe after a restart runs before the timed calls


def queued(config: str, calls: int = 100, depth: int = 2, flags: int = 0, device: int = 0) -> dict:
    """display() calls that do not wait for their frame, as a GL program's do (glutSwapBuffers returns
    while the driver holds a few frames): pt_render_frame_async per call, pt_synchronize every `depth`
    calls (a queue of at most `depth` frames). Reports the mean wall time per call."""
    cfg, tris, nodes, hdr = scenes.build_config(config)
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, device=device,
                  flags=flags) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        f = 0
        for _ in range(PROBE_FRAMES + 10):
            r.render_frame(eye, rot, f, sync=False)
            f += 1
        r.synchronize()
        r.reset_stats()
        t0 = time.perf_counter()
        for k in range(calls):
            r.render_frame(eye, rot, f, sync=False)
            f += 1
            if (k + 1) % depth == 0:
                r.synchronize()
        r.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / calls
        st = r.stats()
    rays = st.rays / max(st.frames, 1)
    return {"config": config, "calls": calls, "queue_depth": depth, "ms_per_call": round(ms, 4),
            "mrays_per_s": round(rays / (ms * 1e-3) / 1e6, 1),
            "frame_kernel": "path regeneration" if st.regen else "lock-step megakernel"}


def per_call(config: str, calls: int = 100, warmup: int = 10, flags: int = 0, device: int = 0,
             scene=None, split: bool = False) -> dict:
    cfg, tris, nodes, hdr = scene if scene is not None else scenes.build_config(config)
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, device=device,
                  flags=flags) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        f = 0
        for _ in range(PROBE_FRAMES):
            r.render_frame(eye, rot, f, sync=False)
            f += 1
        r.synchronize()
        for _ in range(warmup):
            r.render_frame(eye, rot, f)
            f += 1
        r.reset_stats()
        if os.environ.get("PER_CALL_TRACE"):  # a PT_WAVE_TRACE build records the timed calls' waves only
            os.environ["PT_WAVE_TRACE_FILE"] = os.environ["PER_CALL_TRACE"]
        ms, issue = [], []
        for _ in range(calls):
            t0 = time.perf_counter()
            if split:  # the call's two halves: issuing the frame, then waiting for it (pt_synchronize)
                r.render_frame(eye, rot, f, sync=False)
                issue.append(1e3 * (time.perf_counter() - t0))
                r.synchronize()
            else:
                r.render_frame(eye, rot, f)
            ms.append(1e3 * (time.perf_counter() - t0))
            f += 1
        st = r.stats()
    ms.sort()
    med = statistics.median(ms)
    rays = st.rays / max(st.frames, 1)
    extra = {"issue_ms_median": round(statistics.median(issue), 4)} if split else {}
    return {**extra, "config": config, "calls": calls, "warmup": warmup, "median_ms": round(med, 4),
            "p10_ms": round(ms[len(ms) // 10], 4), "p90_ms": round(ms[(9 * len(ms)) // 10], 4),
            "min_ms": round(ms[0], 4), "kernel_ms": round(st.kernel_ms_total / max(st.launches, 1), 4),
            "rays_per_frame": int(rays), "mrays_per_s": round(rays / (med * 1e-3) / 1e6, 1),
            "frame_kernel": "path regeneration" if st.regen else "lock-step megakernel"}


def analyze(trace_dir: str, last: int = 60):
    """A rocprofv3 --kernel-trace of this script: per kernel name, the median duration over the last
    `last` calls, and per call the span from its first kernel's start to its last kernel's end and
    the idle gap before the next call's first kernel (the host's return, sync and next launch)."""
    import csv
    import glob
    rows = []
    for fn in glob.glob(str(Path(trace_dir) / "**" / "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # a call = a maximal run of kernels separated by less than 20 us (calls are separated by the sync)
    calls, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(x[1] for x in cur) > 20_000:
            calls.append(cur)
            cur = [r]
        else:
            cur.append(r)
    calls.append(cur)
    calls = calls[-last:]
    by = {}
    for c in calls:
        for s, e, n in c:
            by.setdefault(n.split("(")[0][:80], []).append((e - s) / 1e3)
    out = {"calls": len(calls),
           "span_us_median": statistics.median((max(x[1] for x in c) - c[0][0]) / 1e3 for c in calls),
           "gap_us_median": statistics.median((calls[i + 1][0][0] - max(x[1] for x in calls[i])) / 1e3
                                              for i in range(len(calls) - 1)),
           "kernels": {k: {"n": len(v), "median_us": round(statistics.median(v), 1)} for k, v in by.items()}}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c2", "c4"])
    ap.add_argument("--calls", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--analyze", default=None, help="a rocprofv3 kernel-trace directory of this script")
    ap.add_argument("--split", action="store_true", help="time the issue and the wait of each call apart")
    ap.add_argument("--queue", type=int, default=0, help="calls that wait only every QUEUE frames (queued())")
    a = ap.parse_args()
    if os.environ.get("PT_VARIANT"):  # an in-tree diagnostics / tuning build (tools/tune.py --build)
        from opengl_ray_tracing_amd import _native
        _native.use_variant(os.environ["PT_VARIANT"])
    if a.analyze:
        analyze(a.analyze)
        return
    for c in a.configs:
        if a.queue:
            print(json.dumps(queued(c, a.calls, a.queue, a.flags)), flush=True)
        else:
            print(json.dumps(per_call(c, a.calls, a.warmup, a.flags, split=a.split)), flush=True)


if __name__ == "__main__":
    main()
