"""Ragged and degenerate inputs on the default frame paths, against the oracle bit for bit:
images smaller than one 8x8 wave tile or one pixel wide, rendered as a stream of frames
(pt_render_frames_async: batched launches, the path-regeneration kernel for Lambert and MIS at
2 bounces, the camera-ray pass) and as synchronous display() calls (pt_render_frame: the
lock-step megakernel), and a scene of a single triangle (a root that is a leaf).

Reference: IS main.cpp:659-709 (the frame loop), IS pass1.fsh:846-871 (one sample per pixel and
the running mean), OpenglRayTracing/main.cpp:430-551 (a one-triangle tree is one leaf).
"""
import numpy as np
import pytest

import oracle
from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
from opengl_ray_tracing_amd.scene import Material, Scene

pytestmark = pytest.mark.gpu

FRAMES = 4


def render_both(w, h, integrator, tris, nodes, hdr, eye, rot, max_bounce=2):
    with Renderer(w, h, integrator, max_bounce=max_bounce) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        r.render_frames(eye, rot, 0, FRAMES)
        r.synchronize()
        streamed = r.accum().copy()
    with Renderer(w, h, integrator, max_bounce=max_bounce) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(FRAMES):
            r.render_frame(eye, rot, f)
        called = r.accum().copy()
    o = oracle.Oracle(tris, nodes, hdr)
    acc = np.zeros((h, w, 4), np.float32)
    for f in range(FRAMES):
        acc, _ = o.render(w, h, integrator, f, eye, rot, accum=acc, max_bounce=max_bounce)
    return streamed, called, acc


@pytest.mark.parametrize("w,h", [(1, 1), (5, 3), (8, 1), (1, 9), (33, 31)])
@pytest.mark.parametrize("integrator", ["lambert", "mis"])
def test_tiny_images_equal_oracle(w, h, integrator):
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    streamed, called, ref = render_both(w, h, integrator, tris, nodes, hdr, eye, rot)
    assert np.isfinite(ref).all()
    assert np.array_equal(streamed, ref)
    assert np.array_equal(called, ref)


def test_single_triangle_scene_equals_oracle():
    s = Scene()
    v = np.array([[-1.0, -1.0, 0.0], [1.0, -1.0, 0.0], [0.0, 1.0, 0.0]], np.float32)
    s.add_mesh(v, np.array([[0, 1, 2]], np.int32), Material(baseColor=(0.8, 0.6, 0.4)))
    s.build_bvh("sah", 8)
    tris, nodes = s.encode()
    assert tris.shape[0] == 1
    cfg, _, _, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(15.0, 10.0, 3.0)
    for integrator in ("lambert", "mis"):
        streamed, called, ref = render_both(48, 40, integrator, tris, nodes, hdr, eye, rot)
        assert np.isfinite(ref).all()
        assert np.array_equal(streamed, ref) and np.array_equal(called, ref), integrator


@pytest.mark.parametrize("integrator", ["lambert", "mis"])
def test_screen_tile_ranks_without_tiles(integrator):
    """More ranks than 32x32 screen tiles (a 40x40 window split 8 ways: 4 tiles): the ranks that own
    no tile render nothing, without error; the others' tiles equal the oracle's image."""
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    w = h = 40
    o = oracle.Oracle(tris, nodes, hdr)
    ref = np.zeros((h, w, 4), np.float32)
    for f in range(FRAMES):
        ref, _ = o.render(w, h, integrator, f, eye, rot, accum=ref, max_bounce=2)
    world = 8
    covered = np.zeros((h, w), bool)
    for rank in range(world):
        with Renderer(w, h, integrator, max_bounce=2, tile_rank=rank, tile_world=world) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            r.render_frames(eye, rot, 0, FRAMES - 1)
            r.render_frame(eye, rot, FRAMES - 1)
            a = r.accum()
            n = r.owned_pixel_count()
        mine = np.zeros((h, w), bool)
        owned = range(rank, 4, world)  # shard tiles t (row-major, 2 x 2 of them)
        for t in owned:
            ty, tx = divmod(t, 2)
            mine[32 * ty:32 * ty + 32, 32 * tx:32 * tx + 32] = True
        assert n == 32 * 32 * len(owned)  # packed slots: whole shard tiles
        assert np.array_equal(a[mine], ref[mine])
        assert not a[~mine].any()
        covered |= mine
    assert covered.all()
