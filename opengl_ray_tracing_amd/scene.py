"""Host scene preparation: the reference's host surface (OpenglRayTracing/main.cpp,
ImportanceSampling_LowDiscrepancySequence/main.cpp, hdrloader.cpp), exposed
from libpt.so's C ABI (include/pt_scene.h).

Names follow the reference: ``Material`` (main.cpp:27-42), ``Scene.read_obj``
(readObj, :261-372), ``Scene.build_bvh`` (buildBVH / buildBVHwithSAH, :376-551),
``Scene.encode`` (Triangle_encoded / BVHNode_encoded, :687-716),
``get_transform_matrix`` (:242-258), ``orbit_camera`` (display() camera,
:569-573), ``load_hdr`` (HDRLoader::load) and ``calculate_hdr_cache``
(IS main.cpp:555-652).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _native

BVH_BUILDERS = {"sah": 0, "reference": 0, "median": 1, "fixed_sah": 2, "binned": 3}


@dataclass
class Material:
    """Material of OpenglRayTracing/main.cpp:27-42 (same defaults)."""
    emissive: Sequence[float] = (0.0, 0.0, 0.0)
    baseColor: Sequence[float] = (1.0, 1.0, 1.0)
    subsurface: float = 0.0
    metallic: float = 0.0
    specular: float = 0.0
    specularTint: float = 0.0
    roughness: float = 0.0
    anisotropic: float = 0.0
    sheen: float = 0.0
    sheenTint: float = 0.0
    clearcoat: float = 0.0
    clearcoatGloss: float = 0.0
    IOR: float = 1.0
    transmission: float = 0.0

    def _c(self) -> _native.PtMaterial:
        m = _native.PtMaterial()
        m.emissive[:] = [float(x) for x in self.emissive]
        m.baseColor[:] = [float(x) for x in self.baseColor]
        for k in ("subsurface", "metallic", "specular", "specularTint", "roughness", "anisotropic", "sheen",
                  "sheenTint", "clearcoat", "clearcoatGloss", "IOR", "transmission"):
            setattr(m, k, float(getattr(self, k)))
        return m


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_native.c_float_p)


def get_transform_matrix(rotate=(0, 0, 0), translate=(0, 0, 0), scale=(1, 1, 1)) -> np.ndarray:
    """getTransformMatrix (main.cpp:242-258); column-major 4x4 as 16 f32."""
    lib = _native.load()
    out = np.zeros(16, np.float32)
    r = np.asarray(rotate, np.float32)
    t = np.asarray(translate, np.float32)
    s = np.asarray(scale, np.float32)
    lib.pt_transform_matrix(_fp(r), _fp(t), _fp(s), _fp(out))
    return out


def orbit_camera(rotate_angle: float = 0.0, up_angle: float = 0.0, r: float = 4.0):
    """display() camera (main.cpp:569-573): returns (eye[3], cameraRotate[16] column-major)."""
    lib = _native.load()
    eye = np.zeros(3, np.float32)
    rot = np.zeros(16, np.float32)
    lib.pt_orbit_camera(float(rotate_angle), float(up_angle), float(r), _fp(eye), _fp(rot))
    return eye, rot


class Scene:
    """Triangle list + BVH, encoded exactly as the reference uploads it."""

    def __init__(self):
        self._lib = _native.load()
        h = C.c_void_p()
        _native.check(self._lib.pt_scene_create(C.byref(h)), None, "pt_scene_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.pt_scene_destroy(self._h)
            self._h = None

    @property
    def num_triangles(self) -> int:
        return self._lib.pt_scene_num_triangles(self._h)

    @property
    def num_nodes(self) -> int:
        return self._lib.pt_scene_num_nodes(self._h)

    @property
    def depth(self) -> int:
        return self._lib.pt_scene_depth(self._h)

    def read_obj(self, path: str, material: Material, trans=None, smooth_normal: bool = True):
        m = material._c()
        t = None if trans is None else np.ascontiguousarray(trans, np.float32)
        rc = self._lib.pt_scene_read_obj(self._h, str(path).encode(), C.byref(m), None if t is None else _fp(t),
                                         int(smooth_normal))
        _native.check(rc, None, f"readObj({path})")

    def read_obj_text(self, text: str, material: Material, trans=None, smooth_normal: bool = True):
        m = material._c()
        t = None if trans is None else np.ascontiguousarray(trans, np.float32)
        rc = self._lib.pt_scene_read_obj_text(self._h, text.encode(), C.byref(m), None if t is None else _fp(t),
                                              int(smooth_normal))
        _native.check(rc, None, "readObj(text)")

    def add_mesh(self, vertices: np.ndarray, indices: np.ndarray, material: Material, trans=None,
                 smooth_normal: bool = True):
        """readObj's normalise/transform/normal pipeline on parsed arrays."""
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 3)
        i = np.ascontiguousarray(indices, np.int32).reshape(-1, 3)
        m = material._c()
        t = None if trans is None else np.ascontiguousarray(trans, np.float32)
        rc = self._lib.pt_scene_add_mesh(self._h, _fp(v), v.shape[0], i.ctypes.data_as(_native.c_int_p),
                                         i.shape[0], C.byref(m), None if t is None else _fp(t), int(smooth_normal))
        _native.check(rc, None, "add_mesh")

    def build_bvh(self, builder: str = "sah", leaf_size: int = 8):
        _native.check(self._lib.pt_scene_build_bvh(self._h, BVH_BUILDERS[builder], int(leaf_size)), None,
                      "build_bvh")

    def encode(self):
        """(tris (n,36) f32 Triangle_encoded, nodes (m,12) f32 BVHNode_encoded)."""
        n, m = self.num_triangles, self.num_nodes
        tris = np.zeros((n, 36), np.float32)
        nodes = np.zeros((max(m, 0), 12), np.float32)
        rc = self._lib.pt_scene_encode(self._h, _fp(tris), _fp(nodes) if m else None)
        _native.check(rc, None, "encode")
        return tris, nodes


def load_hdr(path: str) -> np.ndarray:
    """HDRLoader::load (hdrloader.cpp:29-97) -> (h, w, 3) f32, row 0 = first scanline."""
    lib = _native.load()
    w, h = C.c_int(), C.c_int()
    p = _native.c_float_p()
    _native.check(lib.pt_hdr_load(str(path).encode(), C.byref(w), C.byref(h), C.byref(p)), None, f"load_hdr({path})")
    try:
        arr = np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        lib.pt_free(p)
    return arr


def decode_hdr(data: bytes) -> np.ndarray:
    lib = _native.load()
    w, h = C.c_int(), C.c_int()
    p = _native.c_float_p()
    buf = C.create_string_buffer(data, len(data))
    _native.check(lib.pt_hdr_decode(C.cast(buf, C.c_void_p), len(data), C.byref(w), C.byref(h), C.byref(p)), None,
                  "decode_hdr")
    try:
        arr = np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        lib.pt_free(p)
    return arr


def calculate_hdr_cache(hdr: np.ndarray) -> np.ndarray:
    """calculateHdrCache (IS main.cpp:555-652): (h, w, 3) = (sample x, sample y, pdf)."""
    lib = _native.load()
    hdr = np.ascontiguousarray(hdr, np.float32)
    h, w = hdr.shape[:2]
    out = np.zeros((h, w, 3), np.float32)
    _native.check(lib.pt_hdr_cache(_fp(hdr), w, h, _fp(out)), None, "calculate_hdr_cache")
    return out


def write_pfm(path: str, img: np.ndarray) -> None:
    """Linear (h, w, 3|4) f32 image as PFM; row 0 is the bottom (the accumulation's GL order)."""
    lib = _native.load()
    img = np.ascontiguousarray(img, np.float32)
    h, w, c = img.shape
    _native.check(lib.pt_image_write_pfm(str(path).encode(), _fp(img), w, h, c), None, f"write_pfm({path})")


def write_png(path: str, img: np.ndarray, gamma: float = 2.2, flip_rows: bool = True) -> None:
    """8-bit RGB PNG as BasicRayTracingWithC++'s imshow (main.cpp:169-190): clamp(pow(v, 1/gamma)*255).
    flip_rows: the accumulation's row 0 is the bottom; the BASIC integrator's is the top (pass False)."""
    lib = _native.load()
    img = np.ascontiguousarray(img, np.float32)
    h, w, c = img.shape
    _native.check(lib.pt_image_write_png(str(path).encode(), _fp(img), w, h, c, float(gamma), int(flip_rows)),
                  None, f"write_png({path})")


def imshow_bytes(image: np.ndarray) -> np.ndarray:
    """BasicRayTracingWithC++'s imshow conversion (main.cpp:183) of its double image:
    (unsigned char)clamp(pow(v, 1.0f / 2.2f) * 255, 0.0, 255.0) -- the exponent is the float
    1/2.2 promoted to double, the cast truncates. (h, w, 3) -> uint8, same row order."""
    e = np.float64(np.float32(1.0) / np.float32(2.2))
    v = np.power(np.asarray(image, np.float64)[..., :3], e) * 255.0
    return np.clip(v, 0.0, 255.0).astype(np.uint8)


def read_pfm(path: str) -> np.ndarray:
    """(h, w, 3) f32 in stored row order (PFM rows run bottom to top)."""
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4", count=w * h * 3)
    return data.reshape(h, w, 3).astype(np.float32)
