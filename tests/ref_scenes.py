"""Inputs of the reference-pinned host tests (test infrastructure).

Each scene is the list of readObj calls a reference main() makes -- OBJ text,
material, getTransformMatrix(rotate, translate, scale), smoothNormal -- with the
missing models (bunny.obj, quad.obj, teapot.obj) replaced by the repository's
deterministic stand-ins written out as OBJ text. The same calls run through
the reference's own readObj / buildBVHwithSAH / buildBVH / encode compiled from
/root/reference (oracle/ref_harness.cpp, tests/golden/make_ref_fixtures.py) and
through libpt.so's pt_scene_* (tests/test_ref_pinned.py).
"""
from __future__ import annotations

import numpy as np

from opengl_ray_tracing_amd import Material, Scene, scenes


def obj_text(v: np.ndarray, idx: np.ndarray, form: str = "plain") -> str:
    """OBJ text of a float32 mesh; every coordinate printed so that it parses back to the same float.
    form: "plain" (f a b c), "vt" (f a/a b/b c/c: 3 slashes), "vtvn" (f a/a/a ...: 6 slashes)."""
    v = np.asarray(v, np.float32).reshape(-1, 3)
    out = [f"v {x:.9g} {y:.9g} {z:.9g}" for x, y, z in v.tolist()]
    if form != "plain":
        out += [f"vt {k / len(v):.6f} 0.5" for k in range(len(v))]
        out += ["vn 0 1 0"]
    for a, b, c in (np.asarray(idx).reshape(-1, 3) + 1).tolist():
        if form == "plain":
            out.append(f"f {a} {b} {c}")
        elif form == "vt":
            out.append(f"f {a}/{a} {b}/{b} {c}/{c}")
        else:
            out.append(f"f {a}/{a}/1 {b}/{b}/1 {c}/{c}/1")
    return "\n".join(out) + "\n"


def _parts():
    bunny = obj_text(*scenes.bunny_standin())
    teapot = obj_text(*scenes.teapot_standin())
    quad = scenes.QUAD_OBJ
    small_v, small_i = scenes.uv_sphere(9, 7, lambda u, v: 1.0 + 0.2 * np.sin(3 * u), center=(0.4, -0.2, 0.1))
    return {
        # OpenglRayTracing/main.cpp:647-670 (bunny stand-in)
        "c2": [
            (bunny, Material(baseColor=(0, 1, 1)), ((0, 0, 0), (0.3, -1.6, 0), (1.5, 1.5, 1.5)), True),
            (quad, Material(baseColor=(0.725, 0.71, 0.68)), ((0, 0, 0), (0, -1.4, 0), (18.83, 0.01, 18.83)), False),
            (quad, Material(baseColor=(1, 1, 1), emissive=(20, 20, 20)), ((0, 0, 0), (0.0, 1.38, -0.0), (0.7, 0.01, 0.7)),
             False),
        ],
        # DisneyBRDF/main.cpp:720-727 (teapot stand-in)
        "c3": [
            (teapot, Material(baseColor=(0.75, 0.7, 0.15), roughness=0.15, metallic=1.0, specular=0.5, clearcoat=1.0),
             ((0, 0, 0), (0, -0.4, 0), (1.75, 1.75, 1.75)), True),
        ],
        # ImportanceSampling_LowDiscrepancySequence/main.cpp:756-771
        "c4": [
            (teapot, Material(roughness=0.5, specular=1.0, metallic=1.0, clearcoat=1.0, clearcoatGloss=0.0,
                              baseColor=(1, 0.73, 0.25)), ((0, 0, 0), (0, -0.5, 0), (0.75, 0.75, 0.75)), True),
            (quad, Material(roughness=0.01, specular=1.0, metallic=0.1, clearcoat=1.0, clearcoatGloss=0.0,
                            baseColor=(1, 1, 1)), ((0, 0, 0), (0, -0.5, 0), (13.0, 0.01, 13.0)), False),
        ],
        # readObj's three face forms (slash counts 0, 3 and 6, OpenglRayTracing/main.cpp:301-313), a rotation
        "objforms": [
            (obj_text(small_v, small_i, "plain"), Material(baseColor=(0.2, 0.4, 0.6)), ((10, 20, 30), (0, 0, 0), (1, 2, 1)),
             True),
            (obj_text(small_v, small_i, "vt"), Material(specular=0.5), ((0, 45, 0), (1, 0, 0), (0.5, 0.5, 0.5)), False),
            (obj_text(small_v, small_i, "vtvn"), Material(sheen=0.3, IOR=1.0), ((0, 0, 90), (0, 1, 0), (1, 1, 3)), True),
        ],
    }


def _c5_parts():
    """scenes.scene_c5: the c3 teapot + the 999,698-triangle heightfield (OBJ text of ~25 MB)."""
    hv, hi = scenes.heightfield(708)
    return _parts()["c3"] + [
        (obj_text(hv, hi), Material(baseColor=(0.6, 0.6, 0.65), roughness=0.4, metallic=0.2, specular=0.5),
         ((0, 0, 0), (0, -1.2, 0), (13.0, 13.0, 13.0)), True)]


SCENES = ("c2", "c3", "c4", "objforms", "c5")
BUILDS = [("c2", "sah"), ("c2", "median"), ("c3", "sah"), ("c4", "sah"), ("objforms", "sah"), ("objforms", "none"),
          ("c5", "sah")]
HDRS = ("peppermint", "san_giuseppe")


BIG = {"c5"}  # fixtures hold digests only


def parts(name: str):
    return _c5_parts() if name == "c5" else _parts()[name]


def material_floats(m: Material):
    return [*m.emissive, *m.baseColor, m.subsurface, m.metallic, m.specular, m.specularTint, m.roughness,
            m.anisotropic, m.sheen, m.sheenTint, m.clearcoat, m.clearcoatGloss]


def build_ours(name: str, builder: str):
    """The same readObj calls and build through libpt.so -> (tris [n,36], nodes [m,12] or None)."""
    s = Scene()
    for text, mat, (r, t, sc), smooth in parts(name):
        s.read_obj_text(text, mat, scenes.get_transform_matrix(r, t, sc), smooth)
    if builder == "none":
        tris, _ = s.encode()
        return tris, None
    s.build_bvh(builder, 8)
    return s.encode()
