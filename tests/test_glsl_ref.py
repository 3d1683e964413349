"""The oracle's restatement of the three pass1.fsh kernels pinned to the reference's own
shader text.

oracle/ref_glsl.cpp compiles IS/D/O pass1.fsh (every token but GLSL's `inout T x`,
written `T& x`) as C++ over the reference's vendored glm, with GLSL's language rules
(float literals, left-to-right arguments, implicit int -> float in built-ins), GL's
NEAREST/CLAMP texture lookup, and the transcendental built-ins bound to
include/pt_fmath.h (the GL driver's are not in the reference). What it computes is
committed under tests/golden/glsl/ (tests/golden/make_glsl_fixtures.py):

  * every shader function on 10^5 random inputs: the oracle's function must give the
    same bits (sha256 of the outputs, NaNs canonical);
  * whole frames through each shader's own main(): O on the bunny scene, D and IS on
    the teapot, IS on the ImportanceSampling scene, 160x90, frames 0..2 of the
    running mean -- the oracle's accumulation must equal it bit for bit.

The GPU kernels are bit-exact against the oracle (tests/test_gpu_*.py), so this pins
them to the reference text too. Where /root/reference is present the comparison is
also run live on fresh inputs."""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
import ref_glsl

GOLD = Path(__file__).resolve().parent / "golden" / "glsl"
FUNCS = json.loads((GOLD / "functions.json").read_text())["functions"]
FRAMES = json.loads((GOLD / "frames.json").read_text())["cases"]


@pytest.mark.parametrize("ent", FUNCS, ids=lambda e: f"{e['fn']}-{e['name'].split()[0]}")
def test_function_equals_reference_text(ent):
    fn = ent["fn"]
    x = ref_glsl.inputs(fn, ent["n"], ent["seed"])
    assert np.array_equal(x[:16].view(np.uint32), np.asarray(ent["head_in"], np.uint32)), "input stream changed"
    y = oracle.glsl_fn(fn, x, ref_glsl.FN_OUT[fn])
    head = ref_glsl.canonical(y[:16])
    assert np.array_equal(head, np.asarray(ent["head_out"], np.uint32)), (ent["name"], head, ent["head_out"])
    assert ref_glsl.digest(y) == ent["digest"], ent["name"]


@pytest.mark.parametrize("case", FRAMES, ids=lambda c: c["case"])
def test_frames_equal_reference_main(case):
    tris, nodes, hdr, cache, eye, rot = ref_glsl.case_inputs(case["config"], tuple(case["camera"]))
    o = oracle.Oracle(tris, nodes, hdr, cache)
    w, h = case["width"], case["height"]
    acc = np.zeros((h, w, 4), np.float32)
    for f in range(case["frames"]):
        acc, c = o.render(w, h, case["integrator"], f, eye, rot, accum=acc)
        assert ref_glsl.digest(acc) == case["digests"][f], (case["case"], f)
    got = ref_glsl.canonical(acc.reshape(-1, 4)[case["sample_index"]])
    assert np.array_equal(got, np.asarray(case["sample_last"], np.uint32))
    assert c.rays > w * h  # the camera sees geometry (bounces traced)


live = pytest.mark.skipif(not ref_glsl.available(), reason="/root/reference absent (fixtures cover it)")


@live
@pytest.mark.parametrize("fn", [f[0] for f in ref_glsl.FUNCS])
def test_function_live_fresh_inputs(fn):
    x = ref_glsl.inputs(fn, 20_000, 7)
    a = ref_glsl.canonical(oracle.glsl_fn(fn, x, ref_glsl.FN_OUT[fn]))
    b = ref_glsl.canonical(ref_glsl.ref_fn(fn, x))
    bad = np.nonzero((a != b).any(1))[0]
    assert bad.size == 0, (ref_glsl.FUNCS[fn][1], bad[:5], x[bad[:2]], a[bad[:2]], b[bad[:2]])


@live
@pytest.mark.parametrize("camera", [(75.0, 5.0, 3.0), (200.0, -10.0, 5.0)])
@pytest.mark.parametrize("which,integ,cfg", [(0, "lambert", "c2"), (1, "disney", "c3"), (2, "mis", "c4")])
def test_frames_live_other_cameras(which, integ, cfg, camera):
    tris, nodes, hdr, cache, eye, rot = ref_glsl.case_inputs(cfg, camera)
    w, h = 96, 64  # another aspect and size
    refs = ref_glsl.ref_frames(which, tris, nodes, hdr, cache, eye, rot, 2, w, h)
    o = oracle.Oracle(tris, nodes, hdr, cache)
    acc = np.zeros((h, w, 4), np.float32)
    for f in range(2):
        acc, _ = o.render(w, h, integ, f, eye, rot, accum=acc)
        assert np.array_equal(ref_glsl.canonical(acc), ref_glsl.canonical(refs[f])), (cfg, camera, f)
