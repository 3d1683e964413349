"""The c5 stress workload (BASELINE configs[4]) at full size on the GPU: the
~1M-triangle heightfield merged with the c3 teapot, 3840x2160, MIS + Sobol,
16 bounces, san_giuseppe env -- the bench's own c5 scene.

Full-size checks are size-independent properties (finite output, alpha = 1,
the runtime tree's image equal to the uploaded tree's bit for bit, the ray
count within the integrator's bound); pixel parity is checked on a seeded
sample of pixels against the CPU restatement (tests/parity.py's bar). A second
case builds the same scene with the reference's SAH builder (z-typo included,
OpenglRayTracing/main.cpp:430-551): a chain-shaped tree more than 2000 levels
deep, so traversal of the uploaded tree runs its HBM overflow stack at scale.
"""
import numpy as np
import pytest

import oracle
import parity
from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_NO_BINS, FLAG_REFERENCE_TREE, Renderer, orbit_camera, scenes

pytestmark = pytest.mark.gpu

FRAMES = 2


def render(cfg, tris, nodes, hdr, flags=0, frames=FRAMES):
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, flags=flags) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(frames):
            r.render_frame(eye, rot, f)
        return r.accum(), r.stats()


def oracle_pixels(cfg, tris, nodes, hdr, px, frames=FRAMES):
    eye, rot = orbit_camera(*cfg.camera)
    orc = oracle.Oracle(tris, nodes, hdr)
    acc = np.zeros((cfg.height, cfg.width, 4), np.float32)
    for f in range(frames):
        acc, _ = orc.render(cfg.width, cfg.height, cfg.integrator, f, eye, rot, accum=acc, pixels=px,
                            max_bounce=cfg.max_bounce, threads=16)
    return acc[px[:, 1], px[:, 0]]


def check_full_frame(cfg, g, st, frames=FRAMES):
    npx = cfg.width * cfg.height
    assert g.shape == (cfg.height, cfg.width, 4)
    assert np.all(np.isfinite(g))
    assert np.all(g[..., 3] == 1.0)
    # every path traces at most 1 camera ray + 2 rays (env shadow + BRDF) per bounce (IS:761-841)
    assert npx * frames <= st.rays <= npx * frames * (1 + 2 * cfg.max_bounce)


def test_c5_full_workload_binned_tree():
    cfg, tris, nodes, hdr = scenes.build_config("c5")
    assert tris.shape[0] > 1_000_000 and (cfg.width, cfg.height, cfg.max_bounce) == (3840, 2160, 16)
    g, st = render(cfg, tris, nodes, hdr)
    check_full_frame(cfg, g, st)
    assert st.regen == 1 and st.waves_per_simd == 4  # the large-scene default (PT_WIDE_SCENE_MB)
    m, sm = render(cfg, tris, nodes, hdr, flags=FLAG_MEGAKERNEL)
    assert sm.regen == 0 and sm.waves_per_simd == 3
    b, sb = render(cfg, tris, nodes, hdr, flags=FLAG_MEGAKERNEL | FLAG_REFERENCE_TREE)
    assert np.array_equal(g, m) and np.array_equal(m, b) and sm.rays == sb.rays
    # the default regen frame takes its camera rays from the camera-ray pass; without it
    # (no bins) the regen kernel traces them itself: the same image and rays
    n, sn = render(cfg, tris, nodes, hdr, flags=FLAG_NO_BINS)
    assert sn.regen == 1 and np.array_equal(g, n) and sn.rays == st.rays
    px = parity.sample_pixels(cfg.width, cfg.height, 2000, seed=5)
    s = parity.assert_parity(g[px[:, 1], px[:, 0]], oracle_pixels(cfg, tris, nodes, hdr, px), "c5/binned")
    print("c5 binned", s, "rays", st.rays)


def test_c5_reference_sah_tree():
    s = scenes.scene_c5()
    s.build_bvh("sah", 8)  # buildBVHwithSAH with its z-typo: depth > 2000
    tris, nodes = s.encode()
    cfg = scenes.CONFIGS["c5"]
    hdr = scenes.load_hdr(scenes.HDR_FILES[cfg.env])
    g, st = render(cfg, tris, nodes, hdr, frames=1)
    check_full_frame(cfg, g, st, frames=1)
    assert st.max_stack > 2000  # the uploaded tree's depth + 1 bounds the traversal stack
    b, sb = render(cfg, tris, nodes, hdr, flags=FLAG_REFERENCE_TREE, frames=1)
    assert np.array_equal(g, b) and st.rays == sb.rays
    px = parity.sample_pixels(cfg.width, cfg.height, 400, seed=9)
    s = parity.assert_parity(g[px[:, 1], px[:, 0]], oracle_pixels(cfg, tris, nodes, hdr, px, frames=1),
                             "c5/reference-sah")
    print("c5 reference-sah", s, "rays", st.rays, "max_stack", st.max_stack)
