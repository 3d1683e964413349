#!/usr/bin/env python3
"""Make tests/golden/glsl/ from the reference's own shader text (TEST INFRASTRUCTURE).

Builds oracle/_ref/libref_glsl.so (oracle/ref_build.py: the three pass1.fsh
fragment shaders compiled as C++ over the vendored glm, oracle/ref_glsl.cpp) and
records what it computes:

  glsl/functions.json   per shader function (tests/ref_glsl.py FUNCS): the sha256
                        of its outputs on FUNC_N inputs drawn from RandomState
                        (frozen stream, so only the seed is stored), plus the first
                        16 input / output rows
  glsl/frames.json      per frame case (tests/ref_glsl.py FRAME_CASES): each frame's
                        accumulation (the shader's own main() over every pixel of a
                        160x90 frame, frames 0..n-1) as a sha256, plus 768 sampled
                        pixels of every frame

The shader text's GLSL transcendentals are glibc's double sin / cos / atan2 / asin /
log / pow rounded to float (oracle/ref_glsl.cpp): the fixtures are the reference's
text evaluated with libm code this repository did not write.

    python tests/golden/make_glsl_fixtures.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import ref_glsl  # noqa: E402

OUT = Path(__file__).resolve().parent / "glsl"
FUNC_N, FUNC_SEED = 100_000, 1
SAMPLES = 768  # sampled pixels per frame (of 14 400)


def main():
    if not ref_glsl.available():
        raise SystemExit("the reference is not present: fixtures cannot be regenerated here")
    OUT.mkdir(exist_ok=True)
    funcs = []
    for fn, name, lines in ref_glsl.FUNCS:
        x = ref_glsl.inputs(fn, FUNC_N, FUNC_SEED)
        y = ref_glsl.ref_fn(fn, x)
        funcs.append({"fn": fn, "name": name, "reference": lines, "n": FUNC_N, "seed": FUNC_SEED,
                      "digest": ref_glsl.digest(y), "head_in": x[:16].view(np.uint32).tolist(),
                      "head_out": ref_glsl.canonical(y[:16]).tolist()})
        print(fn, name, funcs[-1]["digest"][:12])
    (OUT / "functions.json").write_text(json.dumps({"generator": "oracle/ref_glsl.cpp ref_glsl_fn", "functions": funcs}) + "\n")
    frames = []
    for name, which, integ, cfg, cam, nf in ref_glsl.FRAME_CASES:
        tris, nodes, hdr, cache, eye, rot = ref_glsl.case_inputs(cfg, cam)
        outs = ref_glsl.ref_frames(which, tris, nodes, hdr, cache, eye, rot, nf)
        rng = np.random.default_rng(3)
        idx = rng.choice(ref_glsl.FRAME_W * ref_glsl.FRAME_H, SAMPLES, replace=False)
        frames.append({"case": name, "shader": which, "integrator": integ, "config": cfg, "camera": list(cam),
                       "frames": nf, "width": ref_glsl.FRAME_W, "height": ref_glsl.FRAME_H,
                       "digests": [ref_glsl.digest(o) for o in outs], "sample_index": idx.tolist(),
                       "sample_last": ref_glsl.canonical(outs[-1].reshape(-1, 4)[idx]).tolist(),
                       # every frame's sampled pixels, for the GPU's tolerance check (tests/test_gpu_libm_pin.py)
                       "sample_frames": [ref_glsl.canonical(o.reshape(-1, 4)[idx]).tolist() for o in outs]})
        print(name, [d[:12] for d in frames[-1]["digests"]])
    (OUT / "frames.json").write_text(json.dumps({"generator": "oracle/ref_glsl.cpp ref_glsl_render", "cases": frames}) + "\n")


if __name__ == "__main__":
    main()
