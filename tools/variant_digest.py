#!/usr/bin/env python3
"""Digest of the accumulation a tuning build renders, to check a variant bit-exact
against the default build before timing it (tools/tune.py):

    python tools/variant_digest.py base lpf --config c4 --frames 3

Each variant renders in its own process (one library per process); prints one
JSON line per variant and exits 1 if the digests differ.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(variant: str, config: str, frames: int, flags: int) -> None:
    from opengl_ray_tracing_amd import _native
    if variant != "base":
        _native.use_variant(variant)
    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    cfg, tris, nodes, hdr = scenes.build_config(config)
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, flags=flags) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(frames):
            r.render_frame(eye, rot, f)
        acc = r.accum()
        st = r.stats()
    print(json.dumps({"variant": variant, "config": config, "frames": frames,
                      "sha256": hashlib.sha256(acc.tobytes()).hexdigest(), "rays": st.rays}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--config", default="c4")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.variants[0], a.config, a.frames, a.flags)
        return
    digests = []
    for v in a.variants:
        out = subprocess.run([sys.executable, __file__, v, "--child", "--config", a.config, "--frames",
                              str(a.frames), "--flags", str(a.flags)], capture_output=True, text=True, timeout=600)
        if out.returncode != 0:
            print(json.dumps({"variant": v, "error": out.stderr[-2000:]}), flush=True)
            raise SystemExit(out.returncode)
        line = out.stdout.strip().splitlines()[-1]
        print(line, flush=True)
        digests.append(json.loads(line)["sha256"])
    same = len(set(digests)) == 1
    print(json.dumps({"config": a.config, "bit_exact": same}), flush=True)
    raise SystemExit(0 if same else 1)


if __name__ == "__main__":
    main()
