#!/usr/bin/env python3
"""Headless stand-in for the reference's display loop: render a benchmark
configuration progressively and write the image.

    python tools/render.py --config c2 --frames 64 --out gpurun_out/c2.png   # pass3 tonemap + PNG
    python tools/render.py --config c4 --frames 16 --out gpurun_out/c4.pfm   # linear accumulation

PNG: pass3's tonemap (pass3.fsh:14-24, limit 1.5) then imshow's gamma 2.2
(BasicRayTracingWithC++/main.cpp:169-190); the BASIC config skips the tonemap
like the reference CPU tracer. PFM: the linear running mean.
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/render.png")
    ap.add_argument("--builder", default=None)
    ap.add_argument("--flags", type=int, default=0)
    a = ap.parse_args()
    import numpy as np

    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes, write_pfm, write_png
    cfg, tris, nodes, hdr = scenes.build_config(a.config, a.builder)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    basic = cfg.integrator == "basic"
    kw = dict(basic_samples=a.frames) if basic else {}
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, flags=a.flags, **kw) as r:
        if basic:
            r.upload_shapes(scenes.cornell_shapes())
            eye, rot = np.zeros(3, np.float32), np.eye(4, dtype=np.float32)
        else:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            eye, rot = orbit_camera(*cfg.camera)
        t0 = time.perf_counter()
        for f in range(a.frames):
            r.render_frame(eye, rot, f, sync=False)
        r.synchronize()
        dt = time.perf_counter() - t0
        st = r.stats()
        if a.out.endswith(".pfm"):
            write_pfm(a.out, r.accum())
        elif basic:  # imshow of the reference's double image (main.cpp:169-190)
            from PIL import Image

            from opengl_ray_tracing_amd.scene import imshow_bytes
            Image.fromarray(imshow_bytes(r.basic_image())).save(a.out)
        else:
            write_png(a.out, r.tonemap(1.5), 2.2, flip_rows=True)
    print(f"{a.config}: {a.frames} frames in {dt * 1e3:.1f} ms, {st.rays / dt / 1e6:.1f} Mrays/s -> {a.out}")


if __name__ == "__main__":
    main()
