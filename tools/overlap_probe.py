#!/usr/bin/env python3
"""How much would overlapping consecutive frames gain? K independent contexts
(each its own HIP stream and accumulation) render the same workload with their
frames interleaved asynchronously, so the GPU can run one context's frame
during another's tail; prints frames per second of K contexts against one.

    python tools/overlap_probe.py --config c2 --k 1 2 3 4 [--tile-world 8]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--k", type=int, nargs="*", default=[1, 2, 3, 4])
    ap.add_argument("--tile-world", type=int, default=1)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--variant", default=None, help="an in-tree tuning build (tools/tune.py --build)")
    a = ap.parse_args()
    if a.variant:
        from opengl_ray_tracing_amd import _native
        _native.use_variant(a.variant)
    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    cfg, tris, nodes, hdr = scenes.build_config(a.config)
    eye, rot = orbit_camera(*cfg.camera)
    base = None
    for k in a.k:
        rs = [Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, tile_world=a.tile_world)
              for _ in range(k)]
        for r in rs:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for f in range(20):
                r.render_frame(eye, rot, f, sync=False)
            r.synchronize()
        t0 = time.perf_counter()
        for f in range(a.frames):
            for r in rs:
                r.render_frame(eye, rot, 20 + f, sync=False)
        for r in rs:
            r.synchronize()
        dt = time.perf_counter() - t0
        ms_per_frame = 1e3 * dt / (a.frames * k)
        base = base or ms_per_frame
        print(json.dumps({"variant": a.variant, "config": a.config, "tile_world": a.tile_world, "k": k,
                          "ms_per_frame": round(ms_per_frame, 4), "speedup": round(base / ms_per_frame, 3)}), flush=True)
        for r in rs:
            r.close()


if __name__ == "__main__":
    main()
