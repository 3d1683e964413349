"""GPU edge cases against the CPU restatement (bit-exact): a root that is a
leaf, axis-aligned and degenerate rays, resolutions that are not multiples of
the 8x8 wave tile, no environment map, maximum bounce counts, and leaves of
the maximum size."""
import numpy as np
import pytest

import oracle
from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes

pytestmark = pytest.mark.gpu


def one_triangle():
    t = np.zeros((1, 36), np.float32)
    t[0, 0:9] = [-1, -1, 0, 1, -1, 0, 0, 1, 0]
    t[0, 9:18] = [0, 0, 1] * 3
    t[0, 21:24] = [0.8, 0.6, 0.4]
    dummy = np.array([255, 128, 0, 30, 0, 0, 1, 1, 0, 0, 1, 0], np.float32)
    root = np.array([0, 0, 0, 1, 0, 0, -1, -1, 0, 1, 1, 0], np.float32)  # leaf: n = 1, index 0
    return t, np.stack([dummy, root])


def special_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-2, 2, (n, 3))
    d = rng.normal(size=(n, 3))
    k = n // 4
    d[:k, 0] = 0.0          # zero components: 1/d = inf, 0 * inf = NaN in the slab test
    d[k:2 * k, 1:] = 0.0    # axis-aligned
    d[2 * k:3 * k, 2] = 0.0  # parallel to z = const planes
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-30)
    return np.concatenate([o, d], 1).astype(np.float32)


def test_root_leaf_and_special_rays():
    tris, nodes = one_triangle()
    rays = special_rays(4096, 3)
    rays[:64, 0:3] = [0, 0, -3]
    rays[:64, 3:6] = [0, 0, 1]  # straight hits
    with Renderer(8, 8) as r:
        r.upload_scene(tris, nodes)
        t, tri = r.trace_closest(rays)
    t_o, tri_o, _ = oracle.Oracle(tris, nodes).trace_closest(rays)
    assert np.all(tri[:64] == 0)
    assert np.array_equal(tri, tri_o) and np.array_equal(t, t_o)


def test_special_rays_on_a_real_tree():
    cfg, tris, nodes, hdr = scenes.build_config("c4")
    rays = special_rays(20000, 5)
    with Renderer(8, 8) as r:
        r.upload_scene(tris, nodes)
        t, tri = r.trace_closest(rays)
    t_o, tri_o, _ = oracle.Oracle(tris, nodes).trace_closest(rays)
    assert (tri_o >= 0).mean() > 0.05
    assert np.array_equal(tri, tri_o) and np.array_equal(t, t_o)


@pytest.mark.parametrize("integrator,max_bounce,env", [("lambert", 0, True), ("disney", 1, False),
                                                        ("mis", 16, True), ("mis", 3, False)])
def test_odd_resolution_bounces_and_env(integrator, max_bounce, env):
    cfg, tris, nodes, hdr = scenes.build_config("c3")
    hdr = hdr if env else None
    w, h = 333, 197  # not multiples of the 8x8 wave tile or the 32x32 shard tile
    eye, rot = orbit_camera(20, 10, 4)
    with Renderer(w, h, integrator, max_bounce=max_bounce) as r:
        r.upload_scene(tris, nodes)
        if env:
            r.upload_env(hdr)
        for f in range(2):
            r.render_frame(eye, rot, f)
        g = r.accum()
    o = oracle.Oracle(tris, nodes, hdr)
    acc = np.zeros((h, w, 4), np.float32)
    for f in range(2):
        acc, _ = o.render(w, h, integrator, f, eye, rot, accum=acc, max_bounce=max_bounce)
    # MIS without an environment divides by pdf_light = 0 (IS:789), as the shader would with an
    # unbound cache texture: NaN pixels in both, so NaNs compare equal here
    assert np.array_equal(g, acc, equal_nan=True)
    if env or integrator != "mis":
        assert np.isfinite(g).all()


def test_max_leaf_size():
    """Leaves of up to 32 triangles (the device encoding's limit; the reference builders use 8)."""
    s = scenes.scene_c2()
    s.build_bvh("binned", 32)
    tris, nodes = s.encode()
    assert nodes[1:, 3].max() > 8
    rays = special_rays(20000, 9)
    eye, _ = orbit_camera(0, 0, 4)
    rays[:10000, 0:3] = eye
    with Renderer(8, 8) as r:
        r.upload_scene(tris, nodes)
        t, tri = r.trace_closest(rays)
    t_o, tri_o, _ = oracle.Oracle(tris, nodes).trace_closest(rays)
    assert np.array_equal(tri, tri_o) and np.array_equal(t, t_o)
