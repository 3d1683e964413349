"""Deterministic synthetic stand-ins for the reference's scenes.

The reference ships no .obj models (bunny.obj, quad.obj, teapot.obj are
referenced at OpenglRayTracing/main.cpp:651-670, DisneyBRDF/main.cpp:727,
ImportanceSampling_LowDiscrepancySequence/main.cpp:763-771 but absent), so
every mesh here is generated procedurally and then fed through the same
readObj pipeline (normalise by the typo'd AABB, transform, normals) with the
same materials and transforms as the reference's main() functions.

Configs (BASELINE.json "configs"):
  c1  BasicRayTracingWithC++ Cornell box, 256x256, 4 spp (BASIC_CPU_COMPAT)
  c2  OpenglRayTracing bunny scene, 1080p, Lambert, 2 bounces, peppermint env
  c3  DisneyBRDF teapot, 1080p, MIS + Sobol, 2 bounces, peppermint env
  c4  ImportanceSampling scene, 1080p, MIS + Sobol, 8 bounces, san_giuseppe env
  c5  ~1M-triangle heightfield + c3 teapot, 4K, 16 bounces (binned-SAH tree)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from .scene import Material, Scene, get_transform_matrix, load_hdr

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
HDR_FILES = {
    # DisneyBRDF/HDR/peppermint_powerplant_4k.hdr (1024x512)
    "peppermint": GOLDEN / "peppermint_powerplant_4k.hdr",
    # TestDemo/assets/HDR/san_giuseppe_bridge_blurred.hdr (2048x1024), stand-in for the
    # missing chinese_garden_2k.hdr (.MISSING_LARGE_BLOBS)
    "san_giuseppe": GOLDEN / "san_giuseppe_bridge_blurred.hdr",
}

# ---------------------------------------------------------------- meshes
QUAD_OBJ = "v -1 0 -1\nv 1 0 -1\nv 1 0 1\nv -1 0 1\nf 1 3 2\nf 1 4 3\n"


def uv_sphere(nu: int, nv: int, radius_fn, center=(0.0, 0.0, 0.0)):
    """Closed UV sphere with pole fans: 2*nu*(nv-1) triangles, no degenerate faces."""
    verts = [(center[0], center[1] + radius_fn(0.0, 0.0), center[2])]
    for j in range(1, nv):
        v = math.pi * j / nv
        for i in range(nu):
            u = 2 * math.pi * i / nu
            r = radius_fn(u, v)
            verts.append((center[0] + r * math.sin(v) * math.cos(u), center[1] + r * math.cos(v),
                          center[2] + r * math.sin(v) * math.sin(u)))
    verts.append((center[0], center[1] - radius_fn(0.0, math.pi), center[2]))
    south = len(verts) - 1

    def ring(j, i):
        return 1 + (j - 1) * nu + (i % nu)

    idx = []
    for i in range(nu):
        idx.append((0, ring(1, i + 1), ring(1, i)))
    for j in range(1, nv - 1):
        for i in range(nu):
            a, b, c, d = ring(j, i), ring(j, i + 1), ring(j + 1, i), ring(j + 1, i + 1)
            idx.append((a, b, d))
            idx.append((a, d, c))
    for i in range(nu):
        idx.append((south, ring(nv - 1, i), ring(nv - 1, i + 1)))
    return np.asarray(verts, np.float32), np.asarray(idx, np.int32)


def revolve(profile, segments: int, cap_bottom=True, cap_top=True):
    """Surface of revolution about +y of a (r, y) profile; fans close the ends."""
    prof = list(profile)
    verts, idx = [], []
    for (r, y) in prof:
        for i in range(segments):
            a = 2 * math.pi * i / segments
            verts.append((r * math.cos(a), y, r * math.sin(a)))
    n = len(prof)
    for j in range(n - 1):
        for i in range(segments):
            a = j * segments + i
            b = j * segments + (i + 1) % segments
            c = (j + 1) * segments + i
            d = (j + 1) * segments + (i + 1) % segments
            idx.append((a, d, b))
            idx.append((a, c, d))
    if cap_bottom:
        verts.append((0.0, prof[0][1], 0.0))
        cb = len(verts) - 1
        for i in range(segments):
            idx.append((cb, i, (i + 1) % segments))
    if cap_top:
        verts.append((0.0, prof[-1][1], 0.0))
        ct = len(verts) - 1
        base = (n - 1) * segments
        for i in range(segments):
            idx.append((ct, base + (i + 1) % segments, base + i))
    return np.asarray(verts, np.float32), np.asarray(idx, np.int32)


def tube(path, radius: float, segments: int):
    """Open tube of circular section along a polyline."""
    pts = np.asarray(path, np.float64)
    verts, idx = [], []
    for k in range(len(pts)):
        t = pts[min(k + 1, len(pts) - 1)] - pts[max(k - 1, 0)]
        t = t / np.linalg.norm(t)
        h = np.array([0.0, 0.0, 1.0]) if abs(t[2]) < 0.9 else np.array([1.0, 0.0, 0.0])
        n1 = np.cross(t, h)
        n1 /= np.linalg.norm(n1)
        n2 = np.cross(t, n1)
        for i in range(segments):
            a = 2 * math.pi * i / segments
            verts.append(pts[k] + radius * (math.cos(a) * n1 + math.sin(a) * n2))
    for k in range(len(pts) - 1):
        for i in range(segments):
            a = k * segments + i
            b = k * segments + (i + 1) % segments
            c = (k + 1) * segments + i
            d = (k + 1) * segments + (i + 1) % segments
            idx.append((a, b, d))
            idx.append((a, d, c))
    return np.asarray(verts, np.float32), np.asarray(idx, np.int32)


def merge(*parts):
    vs, ids, off = [], [], 0
    for v, i in parts:
        vs.append(v)
        ids.append(i + off)
        off += len(v)
    return np.concatenate(vs).astype(np.float32), np.concatenate(ids).astype(np.int32)


def bunny_standin():
    """'Bunny': bumpy sphere r = 1 + 0.05 sin(7u) sin(5v), 50 x 50 UV, 5,000 triangles,
    offset so that after readObj normalisation it rests on the c2 floor."""
    return uv_sphere(50, 51, lambda u, v: 1.0 + 0.05 * math.sin(7 * u) * math.sin(5 * v), center=(0.0, 1.3, 0.0))


def teapot_standin():
    """'Teapot': revolved body + lid knob + spout and handle tubes, ~6.3k triangles."""
    prof = []
    for j in range(40):
        y = j / 39.0
        r = 0.62 * math.sin(math.pi * (0.18 + 0.64 * y)) + 0.2 - 0.12 * y
        prof.append((r, y))
    body = revolve(prof, 64)
    knob = uv_sphere(12, 9, lambda u, v: 0.09, center=(0.0, 1.07, 0.0))
    spout_path = [(0.65 + 0.5 * s, 0.35 + 0.45 * s * s, 0.0) for s in np.linspace(0.0, 1.0, 25)]
    spout = tube(spout_path, 0.09, 12)
    handle_path = [(-0.62 - 0.32 * math.sin(math.pi * s), 0.25 + 0.5 * s, 0.0) for s in np.linspace(0.0, 1.0, 25)]
    handle = tube(handle_path, 0.06, 12)
    return merge(body, knob, spout, handle)


def heightfield(n: int = 708):
    """(n-1)^2 * 2 triangles of y = 0.1 sin(9x) cos(7z) on [-1,1]^2 (n = 708: 999,698)."""
    x = np.linspace(-1.0, 1.0, n, dtype=np.float64)
    X, Z = np.meshgrid(x, x, indexing="xy")
    Y = 0.1 * np.sin(9 * X) * np.cos(7 * Z)
    verts = np.stack([X, Y, Z], -1).reshape(-1, 3).astype(np.float32)
    i = np.arange(n - 1)
    I, J = np.meshgrid(i, i, indexing="xy")
    a = (J * n + I).ravel()
    b = a + 1
    c = a + n
    d = c + 1
    idx = np.empty((2 * a.size, 3), np.int32)
    idx[0::2] = np.stack([a, d, b], -1)
    idx[1::2] = np.stack([a, c, d], -1)
    return verts, idx


# ---------------------------------------------------------------- scenes
def scene_c2() -> Scene:
    """OpenglRayTracing/main.cpp:647-670."""
    s = Scene()
    v, i = bunny_standin()
    s.add_mesh(v, i, Material(baseColor=(0, 1, 1)), get_transform_matrix((0, 0, 0), (0.3, -1.6, 0), (1.5, 1.5, 1.5)),
               True)
    s.read_obj_text(QUAD_OBJ, Material(baseColor=(0.725, 0.71, 0.68)),
                    get_transform_matrix((0, 0, 0), (0, -1.4, 0), (18.83, 0.01, 18.83)), False)
    s.read_obj_text(QUAD_OBJ, Material(baseColor=(1, 1, 1), emissive=(20, 20, 20)),
                    get_transform_matrix((0, 0, 0), (0.0, 1.38, -0.0), (0.7, 0.01, 0.7)), False)
    return s


def scene_c3() -> Scene:
    """DisneyBRDF/main.cpp:720-727 (gold clearcoat teapot)."""
    s = Scene()
    v, i = teapot_standin()
    m = Material(baseColor=(0.75, 0.7, 0.15), roughness=0.15, metallic=1.0, specular=0.5, clearcoat=1.0)
    s.add_mesh(v, i, m, get_transform_matrix((0, 0, 0), (0, -0.4, 0), (1.75, 1.75, 1.75)), True)
    return s


def scene_c4() -> Scene:
    """ImportanceSampling_LowDiscrepancySequence/main.cpp:756-771 (material carried over, as there)."""
    s = Scene()
    v, i = teapot_standin()
    m = Material(roughness=0.5, specular=1.0, metallic=1.0, clearcoat=1.0, clearcoatGloss=0.0,
                 baseColor=(1, 0.73, 0.25))
    s.add_mesh(v, i, m, get_transform_matrix((0, 0, 0), (0, -0.5, 0), (0.75, 0.75, 0.75)), True)
    m.roughness, m.metallic, m.specular, m.baseColor = 0.01, 0.1, 1.0, (1, 1, 1)
    s.read_obj_text(QUAD_OBJ, m, get_transform_matrix((0, 0, 0), (0, -0.5, 0), (13.0, 0.01, 13.0)), False)
    return s


def scene_c5() -> Scene:
    """Stress: ~1M-triangle heightfield merged with the c3 teapot."""
    s = scene_c3()
    v, i = heightfield(708)
    m = Material(baseColor=(0.6, 0.6, 0.65), roughness=0.4, metallic=0.2, specular=0.5)
    s.add_mesh(v, i, m, get_transform_matrix((0, 0, 0), (0, -1.2, 0), (13.0, 13.0, 13.0)), True)
    return s


def cornell_shapes() -> np.ndarray:
    """BasicRayTracingWithC++/main.cpp:306-353 as 24-double shape records (include/pt_scene.h):
    the vec3 fields hold the float values glm stores (vec3 of double literals rounds each to
    float), the material rates and the sphere radius the reference's doubles (:49-59, :130)."""
    RED, GREEN, BLUE = (1, 0.5, 0.5), (0.5, 1, 0.5), (0.5, 0.5, 1)
    YELLOW, CYAN, WHITE = (1.0, 1.0, 0.1), (0.1, 1.0, 1.0), (1, 1, 1)
    recs = []
    f32 = lambda v: np.asarray(v, np.float64).astype(np.float32).astype(np.float64)  # noqa: E731

    def mat(rec, color, emissive=False, spec=0.0, rough=1.0, refr=0.0, angle=1.0, rrough=0.0):
        rec[10:13] = f32(color)
        rec[16] = 1.0 if emissive else 0.0
        rec[17], rec[18], rec[19], rec[20], rec[21] = spec, rough, refr, angle, rrough

    def sphere(o, r, c, **kw):
        rec = np.zeros(24, np.float64)
        rec[0] = 1.0
        rec[1:4] = f32(o)
        rec[22] = r
        mat(rec, c, **kw)
        recs.append(rec)

    def tri(p1, p2, p3, c, **kw):
        rec = np.zeros(24, np.float64)
        p1, p2, p3 = (np.asarray(p, np.float64).astype(np.float32) for p in (p1, p2, p3))
        rec[1:4], rec[4:7], rec[7:10] = p1, p2, p3
        e1, e2 = p2 - p1, p3 - p1
        # glm cross + normalize in f32, the reference's order (main.cpp:85)
        cx = np.float32(e1[1] * e2[2] - e2[1] * e1[2])
        cy = np.float32(e1[2] * e2[0] - e2[2] * e1[0])
        cz = np.float32(e1[0] * e2[1] - e2[0] * e1[1])
        inv = np.float32(1.0) / np.sqrt(np.float32(np.float32(cx * cx + cy * cy) + cz * cz))
        rec[13:16] = (cx * inv, cy * inv, cz * inv)
        mat(rec, c, **kw)
        recs.append(rec)

    sphere((-0.65, -0.7, 0.0), 0.3, GREEN, spec=0.3, rough=0.1)
    sphere((0.0, -0.3, 0.0), 0.4, WHITE, spec=0.3, refr=0.95, angle=0.1)
    sphere((0.65, 0.1, 0.0), 0.3, BLUE, spec=0.3)
    tri((-0.15, 0.4, -0.6), (-0.15, -0.95, -0.6), (0.15, 0.4, -0.6), YELLOW)
    tri((0.15, 0.4, -0.6), (-0.15, -0.95, -0.6), (0.15, -0.95, -0.6), YELLOW)
    tri((0.4, 0.99, 0.4), (-0.4, 0.99, -0.4), (-0.4, 0.99, 0.4), WHITE, emissive=True)
    tri((0.4, 0.99, 0.4), (0.4, 0.99, -0.4), (-0.4, 0.99, -0.4), WHITE, emissive=True)
    tri((1, -1, 1), (-1, -1, -1), (-1, -1, 1), WHITE)
    tri((1, -1, 1), (1, -1, -1), (-1, -1, -1), WHITE)
    tri((1, 1, 1), (-1, 1, 1), (-1, 1, -1), WHITE)
    tri((1, 1, 1), (-1, 1, -1), (1, 1, -1), WHITE)
    tri((1, -1, -1), (-1, 1, -1), (-1, -1, -1), CYAN)
    tri((1, -1, -1), (1, 1, -1), (-1, 1, -1), CYAN)
    tri((-1, -1, -1), (-1, 1, 1), (-1, -1, 1), BLUE)
    tri((-1, -1, -1), (-1, 1, -1), (-1, 1, 1), BLUE)
    tri((1, 1, 1), (1, -1, -1), (1, -1, 1), RED)
    tri((1, -1, -1), (1, 1, 1), (1, 1, -1), RED)
    return np.stack(recs)


def synthetic_env(w: int = 256, h: int = 128, seed: int = 1234) -> np.ndarray:
    """Small deterministic HDR sky (gradient + sun + noise) for fast tests."""
    rng = np.random.default_rng(seed)
    v = (np.arange(h, dtype=np.float32) + 0.5) / h
    u = (np.arange(w, dtype=np.float32) + 0.5) / w
    U, V = np.meshgrid(u, v)
    sky = np.stack([0.4 + 0.6 * (1 - V), 0.5 + 0.5 * (1 - V), 0.8 + 0.4 * (1 - V)], -1)
    sun = 40.0 * np.exp(-((U - 0.3) ** 2 + (V - 0.25) ** 2) / 0.0008)
    img = sky + sun[..., None] * np.array([1.0, 0.9, 0.7]) + 0.05 * rng.random((h, w, 3))
    return img.astype(np.float32)


@dataclass
class Config:
    name: str
    width: int
    height: int
    integrator: str
    max_bounce: int
    env: str | None
    builder: str = "sah"
    camera: tuple = (0.0, 0.0, 4.0)  # rotateAngle, upAngle, r (main.cpp:146-148)
    spp: int = 1
    description: str = ""


CONFIGS = {
    "c1": Config("c1", 256, 256, "basic", 8, None, spp=4,
                 description="BasicRayTracingWithC++ Cornell box, 256x256, 4 spp"),
    "c2": Config("c2", 1920, 1080, "lambert", 2, "peppermint",
                 description="OpenglRayTracing bunny scene (5k tris), 1080p, 1 spp/frame, Lambert"),
    "c3": Config("c3", 1920, 1080, "mis", 2, "peppermint",
                 description="DisneyBRDF teapot + HDR env, 1080p, MIS + Sobol"),
    "c4": Config("c4", 1920, 1080, "mis", 8, "san_giuseppe",
                 description="ImportanceSampling scene, 1080p, 8 bounces"),
    "c5": Config("c5", 3840, 2160, "mis", 16, "san_giuseppe", builder="binned",
                 description="~1M-triangle heightfield + teapot, 4K, 16 bounces"),
}

SCENE_BUILDERS = {"c2": scene_c2, "c3": scene_c3, "c4": scene_c4, "c5": scene_c5}


def build_config(name: str, builder: str | None = None):
    """-> (config, tris, nodes, hdr or None)"""
    cfg = CONFIGS[name]
    if cfg.integrator == "basic":
        return cfg, cornell_shapes(), None, None
    s = SCENE_BUILDERS[name]()
    s.build_bvh(builder or cfg.builder, 8)
    tris, nodes = s.encode()
    hdr = load_hdr(HDR_FILES[cfg.env]) if cfg.env else None
    return cfg, tris, nodes, hdr
