#!/usr/bin/env python3
"""Per-rank cost of screen-tile sharding, measured on one GPU: for each world
size W, every rank's context (tile_rank r, tile_world W) renders its tiles of
the config's frames alone on the device; prints each rank's mean kernel ms and
wall ms per frame. The slowest rank bounds a W-GPU frame (plus the gather).

    python tools/shard_probe.py --config c2 --worlds 1 2 4 8 [--ranks all|0]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

PROBE = 14


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--worlds", type=int, nargs="*", default=[1, 2, 4, 8])
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--res", type=int, nargs=2, default=None, help="override the config's width height")
    ap.add_argument("--variant", default=None, help="an in-tree tuning build (tools/tune.py --build)")
    a = ap.parse_args()
    if a.variant:
        from opengl_ray_tracing_amd import _native
        _native.use_variant(a.variant)
    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    cfg, tris, nodes, hdr = scenes.build_config(a.config)
    eye, rot = orbit_camera(*cfg.camera)
    if a.res:
        cfg.width, cfg.height = a.res
    for w in a.worlds:
        ranks = range(w) if a.ranks == "all" else [0]
        res = []
        for r in ranks:
            with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, tile_rank=r,
                          tile_world=w, flags=a.flags) as R:
                R.upload_scene(tris, nodes)
                R.upload_env(hdr)
                for f in range(PROBE + 5):
                    R.render_frame(eye, rot, f, sync=False)
                R.synchronize()
                R.reset_stats()
                t0 = time.perf_counter()
                for f in range(a.frames):
                    R.render_frame(eye, rot, PROBE + 5 + f, sync=False)
                R.synchronize()
                wall = (time.perf_counter() - t0) * 1e3 / a.frames
                st = R.stats()
                res.append({"rank": r, "kernel_ms": round(st.kernel_ms_total / st.launches, 4),
                            "wall_ms": round(wall, 4), "rays": st.rays // st.launches,
                            "split_items": st.split_items, "runtime_tree": st.runtime_tree})
        worst = max(x["wall_ms"] for x in res)
        print(json.dumps({"variant": a.variant, "config": a.config, "res": [cfg.width, cfg.height], "flags": a.flags, "world": w,
                          "worst_wall_ms": worst, "ranks": res}), flush=True)


if __name__ == "__main__":
    main()
