"""Renderer: the per-frame loop of the reference (display(), OpenglRayTracing/main.cpp:558-603)
driving the MI355X kernels through the C ABI (include/pt_abi.h).

    r = Renderer(1920, 1080, integrator="lambert")
    r.upload_scene(tris, nodes); r.upload_env(hdr)
    eye, rot = orbit_camera(0, 0, 4)
    for frame in range(n): r.render_frame(eye, rot, frame)
    img = r.accum()          # (h, w, 4) running mean, row 0 = bottom row (GL)

Nothing here has a CPU path: every call goes to libpt.so and raises if the
native library or the GPU is missing.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native

INTEGRATORS = {
    "lambert": 0, "lambert_o": 0,           # OpenglRayTracing/shaders/pass1.fsh
    "disney": 1, "disney_uniform_d": 1,     # DisneyBRDF/shaders/pass1.fsh
    "mis": 2, "disney_mis_sobol_is": 2,     # ImportanceSampling_LowDiscrepancySequence/shaders/pass1.fsh
    "basic": 3, "basic_cpu_compat": 3,      # BasicRayTracingWithC++/main.cpp
}
FLAG_NO_CULL = 0x1
FLAG_CLOSEST_SHADOW = 0x2
FLAG_COUNT_FETCHES = 0x4
FLAG_WAVEFRONT = 0x8  # retired in round 5: pt_create rejects it (include/pt_abi.h)
FLAG_REGEN = 0x10
FLAG_NO_TILE_ORDER = 0x20
FLAG_REFERENCE_TREE = 0x40
FLAG_SERIAL_FRAMES = 0x80
FLAG_NO_BINS = 0x100
FLAG_HOST_ACCEL = 0x200
FLAG_MEGAKERNEL = 0x400
FLAG_PRIMARY_PASS = 0x800
GATHER = {"auto": 0, "copy": 1, "rccl": 2}


@dataclass
class FrameStats:
    rays: int
    node_fetch: int
    tri_fetch: int
    mat_fetch: int
    tex_fetch: int
    kernel_ms: float
    kernel_ms_total: float
    launches: int
    max_stack: int
    split_items: int
    runtime_tree: int
    waves_per_simd: int
    devices: int = 1
    gather: int = 0
    frames_in_flight: int = 1
    upload_ms: float = 0.0
    accel_build_ms: float = 0.0
    accel_device: int = -1
    accel_nodes: int = 0
    accel_depth: int = 0
    regen: int = 0
    frames: int = 0       # frames rendered (a batch launch renders several)
    frame_batch: int = 1  # most frames per launch
    env_compact: int = 0  # the env read from its compact (RGBE) texels (2: and the sample table by rows)
    tree4_nodes: int = 0  # 4-wide runtime-tree nodes


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_native.c_float_p)


def device_count() -> int:
    n = C.c_int()
    _native.load().pt_device_count(C.byref(n))
    return n.value


class Renderer:
    def __init__(self, width: int, height: int, integrator="lambert", max_bounce: int = -1, device: int = 0,
                 tile_rank: int = 0, tile_world: int = 1, tile_size: int = 32, flags: int = 0,
                 basic_samples: int = 128, basic_seed: int = 0, sample_rank: int = 0, sample_world: int = 1,
                 devices=None, gather="auto", frame_batch: int = 0):
        """devices: a list of HIP device ids (2..8, repeats allowed) makes this one context render
        screen tiles on all of them and gather them into the first device's accumulation every
        frame (pt_config.n_devices; gather "auto" / "copy" / "rccl"). frame_batch: most frames per
        launch of render_frames (0 = automatic: 2 x tile_world frames; tile_world on large Disney/MIS
        scenes)."""
        self._lib = _native.load()
        cfg = _native.PtConfig()
        cfg.width, cfg.height = int(width), int(height)
        cfg.integrator = INTEGRATORS[integrator] if isinstance(integrator, str) else int(integrator)
        cfg.max_bounce = int(max_bounce)
        cfg.device_id = int(device)
        cfg.tile_rank, cfg.tile_world, cfg.tile_size = int(tile_rank), int(tile_world), int(tile_size)
        cfg.flags = int(flags)
        cfg.basic_samples = int(basic_samples)
        cfg.basic_seed = int(basic_seed) & 0xFFFFFFFF
        cfg.sample_rank, cfg.sample_world = int(sample_rank), int(sample_world)
        if devices is not None and len(devices) == 1:
            cfg.device_id = int(devices[0])
        if devices is not None and len(devices) > 1:
            cfg.n_devices = len(devices)
            for k, d in enumerate(devices):
                cfg.device_ids[k] = int(d)
            cfg.device_id = int(devices[0])
        cfg.gather = GATHER[gather] if isinstance(gather, str) else int(gather)
        cfg.frame_batch = int(frame_batch)
        from . import HW_QUEUES  # the queues GPU_MAX_HW_QUEUES granted this process (package import)
        cfg.hw_queues = int(HW_QUEUES)
        h = C.c_void_p()
        _native.check(self._lib.pt_create(C.byref(h), C.byref(cfg)), None, "pt_create")
        self._h = h
        self.width, self.height = cfg.width, cfg.height
        self.integrator = cfg.integrator
        self.tile_rank, self.tile_world = cfg.tile_rank, cfg.tile_world
        self.sample_rank, self.sample_world = cfg.sample_rank, cfg.sample_world

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pt_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _ck(self, rc, what):
        _native.check(rc, self._h, what)

    def upload_scene(self, tris: np.ndarray, nodes: np.ndarray):
        t = np.ascontiguousarray(tris, np.float32).reshape(-1, 36)
        n = np.ascontiguousarray(nodes, np.float32).reshape(-1, 12)
        self._ck(self._lib.pt_upload_scene(self._h, _fp(t), t.shape[0], _fp(n), n.shape[0]), "pt_upload_scene")

    def hdr_cache_device(self, hdr: np.ndarray) -> np.ndarray:
        """calculateHdrCache on this context's GPU, (h, w, 3) like scene.calculate_hdr_cache."""
        h = np.ascontiguousarray(hdr, np.float32)
        hh, ww = h.shape[:2]
        out = np.empty((hh, ww, 3), np.float32)
        self._ck(self._lib.pt_hdr_cache_device(self._h, _fp(h), ww, hh, _fp(out)), "pt_hdr_cache_device")
        return out

    def upload_env(self, hdr, cache=None):
        if hdr is None:
            self._ck(self._lib.pt_upload_env(self._h, None, 0, 0, None), "pt_upload_env")
            return
        h = np.ascontiguousarray(hdr, np.float32)
        hh, ww = h.shape[:2]
        c = None if cache is None else np.ascontiguousarray(cache, np.float32)
        self._ck(self._lib.pt_upload_env(self._h, _fp(h), ww, hh, None if c is None else _fp(c)), "pt_upload_env")

    def upload_shapes(self, shapes: np.ndarray):
        """BASIC: n x 24 f64 shape records (scenes.cornell_shapes, include/pt_scene.h)."""
        s = np.ascontiguousarray(shapes, np.float64).reshape(-1, 24)
        self._ck(self._lib.pt_upload_shapes(self._h, s.ctypes.data_as(_native.c_double_p), s.shape[0]),
                 "pt_upload_shapes")

    def basic_image(self) -> np.ndarray:
        """BASIC: the reference's double image (h, w, 3), row 0 = top (BasicRayTracingWithC++/main.cpp:356)."""
        out = np.empty((self.height, self.width, 3), np.float64)
        self._ck(self._lib.pt_download_basic_image(self._h, out.ctypes.data_as(_native.c_double_p)),
                 "pt_download_basic_image")
        return out

    def set_basic_stream(self, stream, offsets):
        """BASIC: replay a recorded randf() stream; offsets (samples, h, w) = where each pixel sample's
        draws start. stream None returns to the per-pixel counter RNG. Returns nothing."""
        if stream is None:
            self._ck(self._lib.pt_set_basic_stream(self._h, None, 0, None, 0), "pt_set_basic_stream")
            return
        st = np.ascontiguousarray(stream, np.float64).reshape(-1)
        off = np.ascontiguousarray(offsets, np.int64).reshape(-1)
        self._keep_stream = (st, off)
        self._ck(self._lib.pt_set_basic_stream(self._h, st.ctypes.data_as(_native.c_double_p), st.size,
                                               off.ctypes.data_as(C.POINTER(C.c_int64)), off.size),
                 "pt_set_basic_stream")

    def set_basic_image(self, img: np.ndarray):
        """BASIC checkpoint restore: the double image (h, w, 3) as basic_image() returned it."""
        a = np.ascontiguousarray(img, np.float64).reshape(self.height, self.width, 3)
        self._ck(self._lib.pt_upload_basic_image(self._h, a.ctypes.data_as(_native.c_double_p)),
                 "pt_upload_basic_image")

    def basic_replay_overruns(self) -> int:
        c = C.c_int64()
        self._ck(self._lib.pt_basic_replay_overruns(self._h, C.byref(c)), "pt_basic_replay_overruns")
        return c.value

    def render_frame(self, eye, camera_rotate, frame_counter: int, download: bool = False, sync: bool = True):
        e = np.ascontiguousarray(eye, np.float32)
        r = np.ascontiguousarray(camera_rotate, np.float32).reshape(16)
        if not sync:
            self._ck(self._lib.pt_render_frame_async(self._h, _fp(e), _fp(r), int(frame_counter) & 0xFFFFFFFF),
                     "pt_render_frame_async")
            return None
        out = np.empty((self.height, self.width, 4), np.float32) if download else None
        self._ck(self._lib.pt_render_frame(self._h, _fp(e), _fp(r), int(frame_counter) & 0xFFFFFFFF,
                                           None if out is None else _fp(out)), "pt_render_frame")
        return out

    def render_frames(self, eye, camera_rotate, frame_counter: int, n: int):
        """n display() calls of one camera (frames frame_counter .. frame_counter + n - 1), rendered
        in batches (pt_render_frames_async; bit for bit n render_frame calls). Asynchronous."""
        e = np.ascontiguousarray(eye, np.float32)
        r = np.ascontiguousarray(camera_rotate, np.float32).reshape(16)
        self._ck(self._lib.pt_render_frames_async(self._h, _fp(e), _fp(r), int(frame_counter) & 0xFFFFFFFF, int(n)),
                 "pt_render_frames_async")

    def trace_closest(self, rays: np.ndarray):
        r = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        n = r.shape[0]
        t = np.empty(n, np.float32)
        tri = np.empty(n, np.int32)
        self._ck(self._lib.pt_trace_closest(self._h, _fp(r), n, _fp(t), tri.ctypes.data_as(_native.c_int_p)),
                 "pt_trace_closest")
        return t, tri

    def build_bvh_device(self, tris: np.ndarray, leaf_size: int = 4):
        """pt_build_bvh_device: the GPU binned-SAH tree over tris (n x 36 f32) in the reference's
        node encoding. Returns (nodes (m x 12 f32, dummy node 0, root 1), order (n int32: input
        index of the triangle at each built position))."""
        t = np.ascontiguousarray(tris, np.float32).reshape(-1, 36)
        n = t.shape[0]
        cap = 2 * n + 2
        nodes = np.zeros((cap, 12), np.float32)
        order = np.empty(n, np.int32)
        m = C.c_int()
        self._ck(self._lib.pt_build_bvh_device(self._h, _fp(t), n, int(leaf_size), _fp(nodes), cap, C.byref(m),
                                               order.ctypes.data_as(_native.c_int_p)), "pt_build_bvh_device")
        return nodes[:m.value].copy(), order

    def accum(self) -> np.ndarray:
        out = np.empty((self.height, self.width, 4), np.float32)
        self._ck(self._lib.pt_download_accum(self._h, _fp(out)), "pt_download_accum")
        return out

    def accum_into(self, dptr: int):
        """Copy the accumulation (H x W x 4 f32) into device memory at dptr (stream-ordered, synchronous)."""
        self._ck(self._lib.pt_download_accum(self._h, C.cast(C.c_void_p(dptr), C.POINTER(C.c_float))),
                 "pt_download_accum")

    def set_accum(self, a: np.ndarray):
        a = np.ascontiguousarray(a, np.float32).reshape(self.height, self.width, 4)
        self._ck(self._lib.pt_upload_accum(self._h, _fp(a)), "pt_upload_accum")

    def clear(self):
        self._ck(self._lib.pt_clear_accum(self._h), "pt_clear_accum")

    def accum_device_ptr(self) -> int:
        p = C.c_void_p()
        self._ck(self._lib.pt_accum_device_ptr(self._h, C.byref(p)), "pt_accum_device_ptr")
        return p.value

    def tonemap(self, limit: float = 1.5, gamma: float = 0.0) -> np.ndarray:
        out = np.empty((self.height, self.width, 3), np.float32)
        self._ck(self._lib.pt_tonemap(self._h, float(limit), float(gamma), _fp(out)), "pt_tonemap")
        return out

    def owned_pixel_count(self, rank=None, world=None) -> int:
        c = C.c_int64()
        rank = self.tile_rank if rank is None else rank
        world = self.tile_world if world is None else world
        self._ck(self._lib.pt_owned_pixel_count(self._h, int(rank), int(world), C.byref(c)), "pt_owned_pixel_count")
        return c.value

    def pack_owned(self, dptr: int):
        self._ck(self._lib.pt_pack_owned(self._h, C.c_void_p(dptr)), "pt_pack_owned")

    def unpack_rank(self, rank: int, world: int, dptr: int):
        self._ck(self._lib.pt_unpack_rank(self._h, int(rank), int(world), C.c_void_p(dptr)), "pt_unpack_rank")

    def unpack_ranks(self, world: int, dpacked):
        """Ranks 1..world-1's packed running means (device pointers, entry 0 ignored) into the
        accumulation, one launch."""
        arr = (C.c_void_p * world)(*[C.c_void_p(int(x)) if x else C.c_void_p() for x in dpacked])
        self._ck(self._lib.pt_unpack_ranks(self._h, int(world), arr), "pt_unpack_ranks")

    def display_pack(self, dptr: int, limit: float = 1.5, gamma: float = 0.0):
        """This rank's owned pixels of the displayed frame (pass3 into an 8-bit window), 3 u8 each."""
        self._ck(self._lib.pt_display_pack(self._h, float(limit), float(gamma), C.c_void_p(dptr)), "pt_display_pack")

    def display_own(self, dimage: int, limit: float = 1.5, gamma: float = 0.0):
        """This rank's tiles (every pixel when tile_world is 1) of the displayed frame into an H x W x 4 u8 image."""
        self._ck(self._lib.pt_display_own(self._h, float(limit), float(gamma), C.c_void_p(dimage)), "pt_display_own")

    def display_unpack(self, world: int, dpacked, dimage: int):
        """Ranks 1..world-1's packed display pixels (device pointers, entry 0 ignored) into the image."""
        arr = (C.c_void_p * world)(*[C.c_void_p(int(x)) if x else C.c_void_p() for x in dpacked])
        self._ck(self._lib.pt_display_unpack(self._h, int(world), arr, C.c_void_p(dimage)), "pt_display_unpack")

    def set_stream(self, stream_ptr: int | None):
        self._ck(self._lib.pt_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None), "pt_set_stream")

    def synchronize(self):
        self._ck(self._lib.pt_synchronize(self._h), "pt_synchronize")

    def stats(self) -> FrameStats:
        s = _native.PtFrameStats()
        self._ck(self._lib.pt_get_stats(self._h, C.byref(s)), "pt_get_stats")
        return FrameStats(s.rays, s.node_fetch, s.tri_fetch, s.mat_fetch, s.tex_fetch, s.kernel_ms,
                          s.kernel_ms_total, s.launches, s.max_stack, s.split_items, s.runtime_tree,
                          s.waves_per_simd, s.devices, s.gather, s.frames_in_flight, s.upload_ms,
                          s.accel_build_ms, s.accel_device, s.accel_nodes, s.accel_depth, s.regen, s.frames,
                          s.frame_batch, s.env_compact, s.tree4_nodes)

    def reset_stats(self):
        self._ck(self._lib.pt_reset_stats(self._h), "pt_reset_stats")
