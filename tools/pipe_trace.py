#!/usr/bin/env python3
"""Timeline of pipelined frames from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace -f csv -d OUT -o run -- python3 tools/pipe_trace.py --child c2 8 60
    python3 tools/pipe_trace.py --analyze OUT

The child renders rank 0's share of an N-way screen-tile split (as tools/shard_time.py) for
K timed frames; the analysis lists, per frame, when its frame kernel, reorder and running-mean
update ran (µs from the first timed frame kernel) and summarises the frame period, the
kernels' durations and overlap, and how long each mix waited after its frame kernel ended.
"""
import csv
import glob
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import os  # noqa: E402

import opengl_ray_tracing_amd  # noqa: E402,F401  (raises GPU_MAX_HW_QUEUES before HIP initialises)


def child(cfg_name, world, frames):
    import os

    import torch  # noqa: F401  (one HIP runtime with torch, as in bench.py)
    from opengl_ray_tracing_amd import _native
    if os.environ.get("PT_VARIANT"):  # an in-tree build variant
        _native.use_variant(os.environ["PT_VARIANT"])
    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    cfg, tris, nodes, hdr = scenes.build_config(cfg_name)
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, tile_rank=0,
                  tile_world=world) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(100):  # the policy probes
            r.render_frame(eye, rot, f, sync=False)
        r.synchronize()
        t0 = time.perf_counter()
        for f in range(100, 100 + frames):
            r.render_frame(eye, rot, f, sync=False)
        r.synchronize()
        print(json.dumps({"config": cfg_name, "world": world, "frames": frames,
                          "ms_per_frame": 1e3 * (time.perf_counter() - t0) / frames}), flush=True)


def analyze(d):
    files = glob.glob(str(Path(d) / "**" / "*kernel_trace.csv"), recursive=True)
    rows = []
    for fn in files:
        with open(fn) as f:
            rows += list(csv.DictReader(f))
    ev = []
    for r in rows:
        name = r.get("Kernel_Name", "")
        kind = ("frame" if ("renderKernel" in name or "regenKernel" in name) else "mix" if "mixKernel" in name
                else "reorder" if "reorderKernel" in name else "primary" if "primaryKernel" in name else None)
        if kind:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r.get("Queue_Id", r.get("Stream_Id", ""))))
    ev.sort()
    frames = [e for e in ev if e[2] == "frame"]
    mixes = [e for e in ev if e[2] == "mix"]
    frames, mixes = frames[-60:], mixes[-60:]
    if not frames:
        print("no frame kernels in", files)
        return
    t0 = frames[0][0]
    print("frame kernels (us): start end dur | queue")
    for s, e, k, q in frames[-12:]:
        print(f"  {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} | q{q}")
    print("mixes (us): start end dur")
    for s, e, k, q in mixes[-12:]:
        print(f"  {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} | q{q}")
    per = (frames[-1][0] - frames[0][0]) / max(1, len(frames) - 1) / 1e3
    dur = sum(e - s for s, e, _, _ in frames) / len(frames) / 1e3
    mdur = sum(e - s for s, e, _, _ in mixes) / max(1, len(mixes)) / 1e3
    # each mix after the frame kernel it follows (the latest frame end before its start)
    waits = []
    for s, e, _, _ in mixes:
        ends = [fe for fs, fe, _, _ in frames if fe <= s]
        if ends:
            waits.append((s - max(ends)) / 1e3)
    # frame kernels running at once, time-averaged over the span of the listed frames
    span0, span1 = frames[0][0], max(e for _, e, _, _ in frames)
    busy = sum(e - s for s, e, _, _ in frames) / max(1, span1 - span0)
    print(json.dumps({"frames_in_flight_avg": round(busy, 2), "frame_period_us": round(per, 1), "frame_kernel_us": round(dur, 1),
                      "mix_us": round(mdur, 1), "mix_start_after_prev_frame_end_us":
                      round(sum(waits) / max(1, len(waits)), 1), "frames": len(frames), "mixes": len(mixes)}))


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        analyze(sys.argv[2])
