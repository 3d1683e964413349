#!/usr/bin/env python3
"""A/B timing of in-tree tuning builds of libpt.so (opengl_ray_tracing_amd/_variants/).

    python tools/tune.py --build w4:PT_MIN_WAVES=4 w5:PT_MIN_WAVES=5   # here (cross-compiles)
    python tools/tune.py --build noslp:+-fno-slp-vectorize             # "+flag" = extra hipcc flag
    python tools/tune.py --variants base w4 w5 --config c2 --rounds 3 # on the GPU box

Each measurement runs in its own process (one library per process); variants
are interleaved round by round. Prints one JSON line per measurement and a
median summary.
"""
from __future__ import annotations

import argparse
import json
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
# hardware queues: the package's policy (12 when GPU_MAX_HW_QUEUES is unset, an explicit value
# respected), as bench.py and the tests
import opengl_ray_tracing_amd  # noqa: E402,F401


def child(variant: str, config: str, frames: int, warmup: int, builder, flags: int = 0, max_bounce=None):
    from opengl_ray_tracing_amd import _native
    if variant != "base":
        _native.use_variant(variant)
    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    cfg, tris, nodes, hdr = scenes.build_config(config, builder)
    eye, rot = orbit_camera(*cfg.camera)
    mb = cfg.max_bounce if max_bounce is None else max_bounce
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=mb, flags=flags) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        r.render_frames(eye, rot, 0, warmup)  # as bench.py: the renderer's frames per launch
        r.synchronize()
        r.reset_stats()
        t0 = time.perf_counter()
        r.render_frames(eye, rot, warmup, frames)
        r.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / frames
        st = r.stats()
    ms = st.kernel_ms_total / st.launches
    # frames in flight overlap their launches: wall ms per frame is the comparable figure
    print(json.dumps({"variant": variant, "flags": flags, "config": config, "max_bounce": mb, "kernel_ms": round(ms, 4),
                      "hw_queues": opengl_ray_tracing_amd.HW_QUEUES,
                      "wall_ms": round(wall, 4),
                      "rays": st.rays // max(st.frames, 1), "frames_per_launch": st.frame_batch,
                      "mrays_s": round(st.rays / (st.kernel_ms_total * 1e-3) / 1e6, 1)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", nargs="*", default=None, help="name:DEF=V,DEF=V ...")
    ap.add_argument("--variants", nargs="*", default=["base"])
    ap.add_argument("--config", default="c2")
    ap.add_argument("--builder", default=None)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=22)  # > the renderer's 19-frame policy probe
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", default=None)
    ap.add_argument("--max-bounce", type=int, default=None)
    ap.add_argument("--flags", type=int, nargs="*", default=[0], help="renderer flags to A/B (e.g. 0 8)")
    a = ap.parse_args()
    if a.child:
        child(a.child, a.config, a.frames, a.warmup, a.builder, a.flags[0], a.max_bounce)
        return
    if a.build is not None:
        from opengl_ray_tracing_amd import _build
        for spec in a.build:
            name, _, defs = spec.partition(":")
            items = [kv for kv in defs.split(",") if kv]
            d = dict(kv.split("=", 1) for kv in items if not kv.startswith("+"))
            flags = [kv[1:] for kv in items if kv.startswith("+")]  # "+-fno-slp-vectorize": an extra hipcc flag
            print("built", _build.build_variant(name, d, flags))
        return
    keys = [(v, f) for v in a.variants for f in a.flags]
    res = {k: [] for k in keys}
    for _ in range(a.rounds):
        for (v, fl) in keys:
            cmd = [sys.executable, __file__, "--child", v, "--config", a.config, "--frames", str(a.frames),
                   "--warmup", str(a.warmup), "--flags", str(fl)] + (["--builder", a.builder] if a.builder else []) \
                + (["--max-bounce", str(a.max_bounce)] if a.max_bounce is not None else [])
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(json.dumps({"variant": v, "flags": fl, "error": out.stderr[-2000:]}), flush=True)
                raise SystemExit(out.returncode)
            line = out.stdout.strip().splitlines()[-1]
            print(line, flush=True)
            res[(v, fl)].append(json.loads(line)["wall_ms"])
    print(json.dumps({"summary": {f"{v}/flags={fl}": {"median_ms": statistics.median(x), "min_ms": min(x)}
                                  for (v, fl), x in res.items()},
                      "config": a.config}), flush=True)


if __name__ == "__main__":
    main()
