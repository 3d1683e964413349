"""Host scene preparation pinned to the reference's own code (CPU tests).

tests/golden/ref/ holds what the reference's readObj, getTransformMatrix,
buildBVHwithSAH (z-typo included), buildBVH, the encode of main() and
calculateHdrCache produce -- compiled from /root/reference itself
(oracle/ref_harness.cpp, tests/golden/make_ref_fixtures.py) -- on the inputs of
tests/ref_scenes.py. libpt.so's pt_scene_* / pt_hdr_cache must equal them bit
for bit, and so must the scenes the benchmark renders (scenes.scene_c*, which
feed the stand-in meshes through pt_scene_add_mesh instead of OBJ text).
"""
import base64
import hashlib
import json
import zlib
from pathlib import Path

import numpy as np
import pytest

import ref_scenes
from opengl_ray_tracing_amd import calculate_hdr_cache, scenes

REF = Path(__file__).resolve().parent / "golden" / "ref"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def unpack(s, shape):
    return np.frombuffer(zlib.decompress(base64.b64decode(s)), np.float32).reshape(shape)


def fixture(name):
    return json.loads((REF / f"{name}.json").read_text())


def first_diff(a, b):
    bad = np.argwhere(np.any(a.view(np.uint32) != b.view(np.uint32), axis=-1))
    return None if len(bad) == 0 else (int(bad[0][0]), a[bad[0][0]].tolist(), b[bad[0][0]].tolist())


@pytest.mark.parametrize("name,builder", [b for b in ref_scenes.BUILDS if b[0] not in ref_scenes.BIG])
def test_scene_build_equals_reference(name, builder):
    f = fixture(f"{name}_{builder}")
    tris, nodes = ref_scenes.build_ours(name, builder)
    assert list(tris.shape) == f["tris_shape"]
    if builder == "none":
        ref_tris = unpack(f["tris_f32_zlib_b64"], f["tris_shape"])
        assert first_diff(tris, ref_tris) is None, first_diff(tris, ref_tris)
    if builder != "none":
        ref_nodes = unpack(f["nodes_f32_zlib_b64"], f["nodes_shape"])
        assert list(nodes.shape) == f["nodes_shape"]
        # node 0 is the reference's dummy node; its index field is uninitialised there
        a, b = nodes.copy(), ref_nodes.copy()
        a[0, 4] = b[0, 4] = 0
        assert first_diff(a, b) is None, first_diff(a, b)
    assert sha(tris) == f["tris_sha256"]


@pytest.mark.parametrize("name", ["c2", "c3", "c4", pytest.param("c5", marks=pytest.mark.slow)])
def test_benchmark_scenes_equal_reference_readobj(name):
    """The bench's scenes (stand-in meshes through pt_scene_add_mesh) are the arrays the
    reference's readObj + buildBVHwithSAH make from the same meshes as OBJ files -- for c5
    the 1M-triangle reference-SAH tree (depth 3855) that tests/test_gpu_c5.py renders."""
    f = fixture(f"{name}_sah")
    s = {"c2": scenes.scene_c2, "c3": scenes.scene_c3, "c4": scenes.scene_c4, "c5": scenes.scene_c5}[name]()
    s.build_bvh("sah", 8)
    tris, nodes = s.encode()
    assert sha(tris) == f["tris_sha256"]
    assert list(nodes.shape) == f["nodes_shape"]
    if name in ref_scenes.BIG:  # digests only (the dummy node's index is 0 on both sides)
        assert sha(nodes) == f["nodes_sha256"]
        return
    nodes[0, 4] = 0
    ref = unpack(f["nodes_f32_zlib_b64"], f["nodes_shape"]).copy()
    ref[0, 4] = 0
    assert np.array_equal(nodes.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("env", ref_scenes.HDRS)
def test_hdr_cache_equals_reference(env):
    f = fixture(f"hdrcache_{env}")
    hdr = np.ascontiguousarray(scenes.load_hdr(scenes.HDR_FILES[env]), np.float32)
    assert sha(hdr) == f["hdr_sha256"]  # the input the reference saw
    cache = calculate_hdr_cache(hdr)
    got = cache.reshape(-1, 3)[np.asarray(f["sample_index"])]
    assert np.array_equal(got, np.asarray(f["sample_values"], np.float32))
    assert sha(np.ascontiguousarray(cache, np.float32)) == f["cache_sha256"]


@pytest.mark.parametrize("env", ref_scenes.HDRS)
def test_hdr_decode_equals_reference(env):
    """The repository's Radiance decoder (csrc/scene.cpp, pt_hdr_decode) gives the texels of the
    reference's own hdrloader.cpp decoders (OpenglRayTracing/hdrloader.cpp:93-191, decrunch /
    oldDecrunch / workOnRGBE, compiled from /root/reference: oracle/ref_hdr.cpp) bit for bit on the
    shipped environment maps."""
    f = fixture(f"hdr_decode_{env}")
    hdr = np.ascontiguousarray(scenes.load_hdr(scenes.HDR_FILES[env]), np.float32)
    assert hdr.shape == (f["height"], f["width"], 3)
    got = hdr.reshape(-1, 3)[np.asarray(f["sample_index"])]
    assert np.array_equal(got, np.asarray(f["sample_values"], np.float32))
    assert sha(hdr) == f["decoded_sha256"]
