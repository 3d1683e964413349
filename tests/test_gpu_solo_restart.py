"""A camera restart issued from a drained GPU (sync, then a mouse move: the reference's
interactive loop, IS main.cpp:659-709) with solo launches on and off (PT_SOLO, read when a
context is created).

A solo launch runs on the caller's stream instead of its slot's; the restart's reset of the
split state and cost estimates (pt_runtime.cpp probePolicy) must be ordered with the launch
that follows it on whichever stream that launch runs (round-5 review). The order and the split
only regroup lanes, so the images and the ray counts of the two runs must be equal bit for bit
(the images' parity with the oracle: tests/test_gpu_parity.py).
"""
import os

import numpy as np
import pytest

from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes

pytestmark = pytest.mark.gpu

W, H = 320, 180


def _run(solo: str, cfg, tris, nodes, hdr):
    old = os.environ.get("PT_SOLO")
    os.environ["PT_SOLO"] = solo
    try:
        r = Renderer(W, H, cfg.integrator, max_bounce=cfg.max_bounce)
    finally:
        if old is None:
            del os.environ["PT_SOLO"]
        else:
            os.environ["PT_SOLO"] = old
    with r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        eye, rot = orbit_camera(*cfg.camera)
        r.render_frames(eye, rot, 0, 24)  # a stream of frames (the policy probe runs here)
        r.synchronize()  # the GPU drains
        images, rays = [], []
        eye2, rot2 = orbit_camera(cfg.camera[0] + 20.0, cfg.camera[1] + 5.0, *cfg.camera[2:])
        for f in range(6):  # the restart and the synchronous calls after it
            r.reset_stats()
            images.append(r.render_frame(eye2, rot2, f, download=True).copy())
            rays.append(r.stats().rays)
        r.render_frames(eye2, rot2, 6, 16)  # and a stream again
        r.synchronize()
        images.append(r.accum().copy())
    return images, rays


@pytest.mark.parametrize("name", ["c4", "c2"])
def test_restart_from_idle_gpu_is_the_same_with_and_without_solo_launches(name):
    cfg, tris, nodes, hdr = scenes.build_config(name)
    a_img, a_rays = _run("1", cfg, tris, nodes, hdr)
    b_img, b_rays = _run("0", cfg, tris, nodes, hdr)
    assert a_rays == b_rays
    for k, (a, b) in enumerate(zip(a_img, b_img)):
        assert np.isfinite(a).all()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (name, k)
