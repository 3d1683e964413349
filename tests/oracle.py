"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference path (oracle/pt_oracle.c). Imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only, and
there only as the checker / the CPU baseline, never as the product path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
LIB_PATH = ROOT / "oracle" / "liboracle.so"

c_float_p = C.POINTER(C.c_float)
c_double_p = C.POINTER(C.c_double)


class OrcScene(C.Structure):
    _fields_ = [("tris", c_float_p), ("nTriangles", C.c_int), ("nodes", c_float_p), ("nNodes", C.c_int),
                ("hdr", c_float_p), ("cache", c_float_p), ("hdrW", C.c_int), ("hdrH", C.c_int),
                ("hdrResolution", C.c_int), ("shapes", c_double_p), ("nShapes", C.c_int)]


class OrcFrame(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("integrator", C.c_int), ("maxBounce", C.c_int),
                ("frameCounter", C.c_uint32), ("eye", C.c_float * 3), ("cameraRotate", C.c_float * 16),
                ("basicSamples", C.c_int), ("basicSeed", C.c_uint32), ("sampleRank", C.c_int),
                ("sampleWorld", C.c_int), ("basicImage", c_double_p)]


class OrcCounters(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("nodes", C.c_uint64), ("tris", C.c_uint64), ("mats", C.c_uint64),
                ("texels", C.c_uint64)]


@dataclass
class Counters:
    rays: int
    nodes: int
    tris: int
    mats: int
    texels: int

    @property
    def bytes(self) -> int:
        """B = 48 F_node + 72 F_tri + 72 F_mat + 12 F_tex."""
        return 48 * self.nodes + 72 * self.tris + 72 * self.mats + 12 * self.texels


_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            from opengl_ray_tracing_amd import _build
            _build.build_oracle()
        lib = C.CDLL(str(LIB_PATH))
        lib.orc_render_pixels.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcFrame), C.POINTER(C.c_int), C.c_int,
                                          c_float_p, C.c_int, C.POINTER(OrcCounters)]
        lib.orc_render_pixels.restype = C.c_int
        lib.orc_trace_closest.argtypes = [C.POINTER(OrcScene), c_float_p, C.c_int, c_float_p, C.POINTER(C.c_int),
                                          C.c_int, C.POINTER(OrcCounters)]
        lib.orc_trace_closest.restype = C.c_int
        lib.orc_wang_hash.argtypes = [C.c_uint32]
        lib.orc_wang_hash.restype = C.c_uint32
        lib.orc_sobol.argtypes = [C.c_uint32, C.c_uint32]
        lib.orc_sobol.restype = C.c_float
        lib.orc_pixel_rng.argtypes = [C.c_int, C.c_int, C.c_uint32, C.c_int, c_float_p]
        lib.orc_pixel_rng.restype = None
        lib.orc_hdr_cache.argtypes = [c_float_p, C.c_int, C.c_int, c_float_p]
        lib.orc_hdr_cache.restype = C.c_int
        lib.orc_basic_serial.argtypes = [C.POINTER(OrcScene), C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_int,
                                         c_double_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                         C.POINTER(OrcCounters)]
        lib.orc_basic_serial.restype = C.c_int
        lib.orc_mt_doubles.argtypes = [C.c_uint32, C.c_int64, c_double_p]
        lib.orc_mt_doubles.restype = C.c_int
        lib.orc_glsl_fn.argtypes = [C.c_int, c_float_p, c_float_p, C.c_int]
        lib.orc_glsl_fn.restype = C.c_int
        _lib = lib
    return _lib


INTEG = {"lambert": 0, "disney": 1, "mis": 2, "basic": 3}


class Oracle:
    """Holds the scene arrays alive while the C structs point at them."""

    def __init__(self, tris=None, nodes=None, hdr=None, cache=None, shapes=None):
        self.lib = load()
        self._keep = []
        s = OrcScene()

        def fp(a):
            if a is None:
                return None
            a = np.ascontiguousarray(a, np.float32)
            self._keep.append(a)
            return a.ctypes.data_as(c_float_p)

        if tris is not None:
            s.tris, s.nTriangles = fp(tris), int(np.asarray(tris).reshape(-1, 36).shape[0])
        if nodes is not None:
            s.nodes, s.nNodes = fp(nodes), int(np.asarray(nodes).reshape(-1, 12).shape[0])
        if hdr is not None:
            h, w = hdr.shape[:2]
            if cache is None:
                cache = hdr_cache(hdr)
            s.hdr, s.cache, s.hdrW, s.hdrH, s.hdrResolution = fp(hdr), fp(cache), w, h, w
        if shapes is not None:
            sh = np.ascontiguousarray(shapes, np.float64).reshape(-1, 24)
            self._keep.append(sh)
            s.shapes, s.nShapes = sh.ctypes.data_as(c_double_p), int(sh.shape[0])
        self.scene = s
        self.basic_image = None  # BASIC: the reference's double image, summed across frames

    def render(self, width, height, integrator, frame, eye=None, rot=None, accum=None, pixels=None,
               max_bounce=-1, threads=8, basic_samples=128, basic_seed=0, sample_rank=0, sample_world=1):
        f = OrcFrame()
        f.width, f.height = width, height
        f.integrator = INTEG[integrator] if isinstance(integrator, str) else integrator
        f.maxBounce = max_bounce
        f.frameCounter = frame & 0xFFFFFFFF
        if eye is not None:
            f.eye[:] = [float(x) for x in eye]
        if rot is not None:
            f.cameraRotate[:] = [float(x) for x in np.asarray(rot).reshape(16)]
        f.basicSamples = basic_samples
        f.basicSeed = basic_seed
        f.sampleRank, f.sampleWorld = sample_rank, sample_world
        if accum is None:
            accum = np.zeros((height, width, 4), np.float32)
        assert accum.dtype == np.float32 and accum.flags.c_contiguous and accum.shape == (height, width, 4)
        if f.integrator == INTEG["basic"]:
            if self.basic_image is None or self.basic_image.shape != (height, width, 3):
                self.basic_image = np.zeros((height, width, 3), np.float64)
            f.basicImage = self.basic_image.ctypes.data_as(c_double_p)
        cnt = OrcCounters()
        if pixels is not None:
            px = np.ascontiguousarray(pixels, np.int32).reshape(-1, 2)
            pp, n = px.ctypes.data_as(C.POINTER(C.c_int)), px.shape[0]
        else:
            pp, n = None, 0
        rc = self.lib.orc_render_pixels(C.byref(self.scene), C.byref(f), pp, n, accum.ctypes.data_as(c_float_p),
                                        threads, C.byref(cnt))
        assert rc == 0, rc
        return accum, Counters(cnt.rays, cnt.nodes, cnt.tris, cnt.mats, cnt.texels)

    def basic_serial(self, width=256, height=256, samples=4, seed=5489, max_depth=8, offsets=False):
        """BasicRayTracingWithC++/main.cpp as shipped (one mt19937 stream, serial loop):
        -> (image (h, w, 3) float64, row 0 = top, offsets (samples, h, w) int64 or None, draws, Counters)"""
        img = np.zeros((height, width, 3), np.float64)
        off = np.zeros((samples, height, width), np.int64) if offsets else None
        nd = C.c_int64()
        cnt = OrcCounters()
        rc = self.lib.orc_basic_serial(C.byref(self.scene), width, height, samples, seed & 0xFFFFFFFF, max_depth,
                                       img.ctypes.data_as(c_double_p),
                                       None if off is None else off.ctypes.data_as(C.POINTER(C.c_int64)),
                                       C.byref(nd), C.byref(cnt))
        assert rc == 0, rc
        return img, off, nd.value, Counters(cnt.rays, cnt.nodes, cnt.tris, cnt.mats, cnt.texels)

    def trace_closest(self, rays, brute=False):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        n = r.shape[0]
        t = np.empty(n, np.float32)
        tri = np.empty(n, np.int32)
        cnt = OrcCounters()
        rc = self.lib.orc_trace_closest(C.byref(self.scene), r.ctypes.data_as(c_float_p), n,
                                        t.ctypes.data_as(c_float_p), tri.ctypes.data_as(C.POINTER(C.c_int)),
                                        int(brute), C.byref(cnt))
        assert rc == 0
        return t, tri, Counters(cnt.rays, cnt.nodes, cnt.tris, cnt.mats, cnt.texels)


def wang_hash(x: int) -> int:
    return load().orc_wang_hash(x & 0xFFFFFFFF)


def sobol(d: int, i: int) -> float:
    return load().orc_sobol(d, i)


def pixel_rng(px, py, frame, n):
    out = np.empty(n, np.float32)
    load().orc_pixel_rng(px, py, frame, n, out.ctypes.data_as(c_float_p))
    return out


def mt_doubles(seed: int, n: int) -> np.ndarray:
    """The reference's randf() stream (BasicRayTracingWithC++/main.cpp:208-214) from std::mt19937(seed)."""
    out = np.empty(n, np.float64)
    assert load().orc_mt_doubles(seed & 0xFFFFFFFF, n, out.ctypes.data_as(c_double_p)) == 0
    return out


def glsl_fn(fn: int, x: np.ndarray, n_out: int) -> np.ndarray:
    """The restatement's function fn (orc_glsl_fn, the layout of tests/ref_glsl.py FUNCS) on rows of x."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros((x.shape[0], n_out), np.float32)
    assert load().orc_glsl_fn(fn, x.ctypes.data_as(c_float_p), out.ctypes.data_as(c_float_p), x.shape[0]) == 0
    return out


def hdr_cache(hdr):
    hdr = np.ascontiguousarray(hdr, np.float32)
    h, w = hdr.shape[:2]
    out = np.zeros((h, w, 3), np.float32)
    assert load().orc_hdr_cache(hdr.ctypes.data_as(c_float_p), w, h, out.ctypes.data_as(c_float_p)) == 0
    return out
