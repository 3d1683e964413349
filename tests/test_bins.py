"""Camera-ray bins are conservative (CPU test of pt_primary.hip's binning rule).

binRect below restates binRectKernel (pt_primary.hip) in numpy float64. For
seeded camera rays of several frames and cameras -- generated with the
reference's ray generation (IS:846-850, float32, as pt_kernels.hip cameraRay)
-- the CPU oracle's brute-force closest hit (hitArray over every triangle,
IS:853-854) must lie in the bin of the ray's 8x8 tile: the rectangle binRect
gives that triangle must contain the tile. (The GPU test
test_camera_bins_equal_bvh_camera_rays checks the images themselves.)
"""
import numpy as np
import pytest

import oracle
from opengl_ray_tracing_amd import orbit_camera, scenes

NEAR_Z, MARGIN = -2.5e-4, 2.0


def bin_rect(tris, eye, cam, w, h):
    """(tx0, ty0, tx1, ty1) per triangle, tx0 > tx1 when it has no bin (binRectKernel)."""
    tilesX, tilesY = (w + 7) // 8, (h + 7) // 8
    R = np.stack([np.asarray(cam, np.float64)[4 * a:4 * a + 3] for a in range(3)])  # rows: c0, c1, c2
    v = tris[:, :9].astype(np.float64).reshape(-1, 3, 3) - np.asarray(eye, np.float64)
    q = np.einsum("ij,tkj->tki", R, v)  # camera space, per vertex
    out = np.zeros((len(tris), 4), np.int64)
    out[:, 0], out[:, 2] = 1, 0
    for i in range(len(tris)):
        pts = []
        for k in range(3):
            a, b = q[i, k], q[i, (k + 1) % 3]
            ain, bin_ = a[2] <= NEAR_Z, b[2] <= NEAR_Z
            if ain:
                pts.append((-1.5 * a[0] / a[2], -1.5 * a[1] / a[2]))
            if ain != bin_:
                s = (NEAR_Z - a[2]) / (b[2] - a[2])
                x, y = a[0] + s * (b[0] - a[0]), a[1] + s * (b[1] - a[1])
                pts.append((-1.5 * x / NEAR_Z, -1.5 * y / NEAR_Z))
        if not pts:
            continue
        X = [(p[0] + 1.0) * 0.5 * w - 0.5 for p in pts]
        Y = [(p[1] + 1.0) * 0.5 * h - 0.5 for p in pts]
        x0, x1, y0, y1 = min(X) - MARGIN, max(X) + MARGIN, min(Y) - MARGIN, max(Y) + MARGIN
        if x1 >= 0 and y1 >= 0 and x0 <= w - 1 and y0 <= h - 1:
            tx0, ty0 = max(0, int(np.floor(x0 / 8))), max(0, int(np.floor(y0 / 8)))
            tx1, ty1 = min(tilesX - 1, int(np.floor(x1 / 8))), min(tilesY - 1, int(np.floor(y1 / 8)))
            if tx0 <= tx1 and ty0 <= ty1:
                out[i] = (tx0, ty0, tx1, ty1)
    return out


def wang(s):
    s = (s ^ np.uint32(61)) ^ (s >> np.uint32(16))
    s = s * np.uint32(9)
    s = s ^ (s >> np.uint32(4))
    s = s * np.uint32(0x27D4EB2D)
    return s ^ (s >> np.uint32(15))


def camera_rays(px, py, frame, eye, cam, w, h):
    """cameraRay (pt_kernels.hip) / IS:73-89, 846-850 in float32."""
    f32 = np.float32
    with np.errstate(over="ignore"):
        seed = (px.astype(np.uint32) * np.uint32(1973) + py.astype(np.uint32) * np.uint32(9277)
                + np.uint32(frame) * np.uint32(26699)) | np.uint32(1)
        s1 = wang(seed)
        s2 = wang(s1)
    r1 = s1.astype(f32) / f32(4294967296.0)
    r2 = s2.astype(f32) / f32(4294967296.0)
    pixx = (2 * px + 1).astype(f32) / f32(w) - f32(1)
    pixy = (2 * py + 1).astype(f32) / f32(h) - f32(1)
    x = pixx + (r1 - f32(0.5)) / f32(w)
    y = pixy + (r2 - f32(0.5)) / f32(h)
    M = np.asarray(cam, f32)
    c0, c1, c2 = M[0:3], M[4:7], M[8:11]
    d = (c0[None] * x[:, None] + c1[None] * y[:, None]) + c2[None] * f32(-1.5)
    d = d / np.sqrt((d * d).sum(1, dtype=f32)).astype(f32)[:, None]
    o = np.repeat(np.asarray(eye, f32)[None], len(px), 0)
    return np.concatenate([o, d], 1).astype(f32)


@pytest.mark.parametrize("name,camera", [("c2", None), ("c2", (35.0, 20.0, 2.5)), ("c4", None),
                                         ("c4", (-60.0, 40.0, 1.2))])
def test_every_hit_triangle_is_in_its_tile_bin(name, camera):
    cfg, tris, nodes, hdr = scenes.build_config(name)
    w, h = 640, 360
    eye, cam = orbit_camera(*(camera or cfg.camera))
    rects = bin_rect(tris, eye, cam, w, h)
    rng = np.random.default_rng(5)
    k = rng.choice(w * h, 6000, replace=False)
    px, py = (k % w).astype(np.int64), (k // w).astype(np.int64)
    orc = oracle.Oracle(tris, nodes)
    checked = 0
    for frame in (0, 1, 7):
        rays = camera_rays(px, py, frame, eye, cam, w, h)
        _, tri, _ = orc.trace_closest(rays, brute=True)
        hit = tri >= 0
        tx, ty = px[hit] // 8, py[hit] // 8
        r = rects[tri[hit]]
        inside = (r[:, 0] <= tx) & (tx <= r[:, 2]) & (r[:, 1] <= ty) & (ty <= r[:, 3])
        assert inside.all(), (name, camera, frame, np.flatnonzero(~inside)[:5])
        checked += int(hit.sum())
    assert checked > 3000
