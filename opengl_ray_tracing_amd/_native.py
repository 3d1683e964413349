"""ctypes binding of libpt.so (include/pt_abi.h + include/pt_scene.h).

The product path has no fallback: if libpt.so is missing or fails to load,
every entry point raises. Build it with ``python -m opengl_ray_tracing_amd._build``
or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

from . import _build

_lib = None

ABI_VERSION = 7  # include/pt_abi.h PT_ABI_VERSION
# an older tuning build (tools/tune.py A/B against a previous round's library) loads when its structs
# match: ABI 7 only added pt_unpack_ranks, which such a build does not have
ABI_STRUCTS_SINCE = 6
c_float_p = C.POINTER(C.c_float)
c_double_p = C.POINTER(C.c_double)
c_int_p = C.POINTER(C.c_int)


class PtConfig(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("integrator", C.c_int), ("max_bounce", C.c_int),
        ("device_id", C.c_int), ("tile_rank", C.c_int), ("tile_world", C.c_int), ("tile_size", C.c_int),
        ("flags", C.c_uint32), ("basic_samples", C.c_int), ("basic_seed", C.c_uint32),
        ("sample_rank", C.c_int), ("sample_world", C.c_int),
        ("n_devices", C.c_int), ("device_ids", C.c_int * 8), ("gather", C.c_int),
        ("frame_batch", C.c_int), ("hw_queues", C.c_int),
    ]


class PtFrameStats(C.Structure):
    _fields_ = [
        ("rays", C.c_uint64), ("node_fetch", C.c_uint64), ("tri_fetch", C.c_uint64),
        ("mat_fetch", C.c_uint64), ("tex_fetch", C.c_uint64), ("kernel_ms", C.c_float),
        ("kernel_ms_total", C.c_float), ("launches", C.c_int), ("max_stack", C.c_int),
        ("split_items", C.c_int), ("runtime_tree", C.c_int),
        ("waves_per_simd", C.c_int), ("devices", C.c_int), ("gather", C.c_int), ("frames_in_flight", C.c_int),
        ("upload_ms", C.c_float), ("accel_build_ms", C.c_float), ("accel_device", C.c_int),
        ("accel_nodes", C.c_int), ("accel_depth", C.c_int), ("regen", C.c_int),
        ("frames", C.c_int64), ("frame_batch", C.c_int), ("env_compact", C.c_int), ("tree4_nodes", C.c_int),
    ]


class PtMaterial(C.Structure):
    _fields_ = [
        ("emissive", C.c_float * 3), ("baseColor", C.c_float * 3),
        ("subsurface", C.c_float), ("metallic", C.c_float), ("specular", C.c_float),
        ("specularTint", C.c_float), ("roughness", C.c_float), ("anisotropic", C.c_float),
        ("sheen", C.c_float), ("sheenTint", C.c_float), ("clearcoat", C.c_float),
        ("clearcoatGloss", C.c_float), ("IOR", C.c_float), ("transmission", C.c_float),
    ]


# name -> (restype, argtypes); every symbol declared in include/pt_abi.h and include/pt_scene.h
SIGNATURES = {
    # pt_abi.h
    "pt_device_count": (C.c_int, [c_int_p]),
    "pt_abi_version": (C.c_int, []),
    "pt_create": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(PtConfig)]),
    "pt_destroy": (None, [C.c_void_p]),
    "pt_last_error": (C.c_char_p, [C.c_void_p]),
    "pt_upload_scene": (C.c_int, [C.c_void_p, c_float_p, C.c_int, c_float_p, C.c_int]),
    "pt_upload_env": (C.c_int, [C.c_void_p, c_float_p, C.c_int, C.c_int, c_float_p]),
    "pt_upload_shapes": (C.c_int, [C.c_void_p, c_double_p, C.c_int]),
    "pt_download_basic_image": (C.c_int, [C.c_void_p, c_double_p]),
    "pt_upload_basic_image": (C.c_int, [C.c_void_p, c_double_p]),
    "pt_set_basic_stream": (C.c_int, [C.c_void_p, c_double_p, C.c_int64, C.POINTER(C.c_int64), C.c_int64]),
    "pt_basic_replay_overruns": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "pt_render_frame": (C.c_int, [C.c_void_p, c_float_p, c_float_p, C.c_uint32, c_float_p]),
    "pt_render_frame_async": (C.c_int, [C.c_void_p, c_float_p, c_float_p, C.c_uint32]),
    "pt_render_frames_async": (C.c_int, [C.c_void_p, c_float_p, c_float_p, C.c_uint32, C.c_int]),
    "pt_trace_closest": (C.c_int, [C.c_void_p, c_float_p, C.c_int, c_float_p, c_int_p]),
    "pt_build_bvh_device": (C.c_int, [C.c_void_p, c_float_p, C.c_int, C.c_int, c_float_p, C.c_int, c_int_p, c_int_p]),
    "pt_download_accum": (C.c_int, [C.c_void_p, c_float_p]),
    "pt_upload_accum": (C.c_int, [C.c_void_p, c_float_p]),
    "pt_clear_accum": (C.c_int, [C.c_void_p]),
    "pt_accum_device_ptr": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "pt_tonemap": (C.c_int, [C.c_void_p, C.c_float, C.c_float, c_float_p]),
    "pt_owned_pixel_count": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int64)]),
    "pt_pack_owned": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pt_unpack_rank": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "pt_unpack_ranks": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "pt_display_pack": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_void_p]),
    "pt_display_own": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_void_p]),
    "pt_display_unpack": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.c_void_p]),
    "pt_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pt_synchronize": (C.c_int, [C.c_void_p]),
    "pt_get_stats": (C.c_int, [C.c_void_p, C.POINTER(PtFrameStats)]),
    "pt_reset_stats": (C.c_int, [C.c_void_p]),
    "pt_fmath_host": (C.c_int, [C.c_int, c_float_p, c_float_p, C.c_int, c_float_p]),
    "pt_fmath_device": (C.c_int, [C.c_void_p, C.c_int, c_float_p, c_float_p, C.c_int, c_float_p]),
    # pt_scene.h
    "pt_material_default": (None, [C.POINTER(PtMaterial)]),
    "pt_scene_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "pt_scene_destroy": (None, [C.c_void_p]),
    "pt_scene_read_obj": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(PtMaterial), c_float_p, C.c_int]),
    "pt_scene_read_obj_text": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(PtMaterial), c_float_p, C.c_int]),
    "pt_scene_add_mesh": (C.c_int, [C.c_void_p, c_float_p, C.c_int, c_int_p, C.c_int, C.POINTER(PtMaterial),
                                    c_float_p, C.c_int]),
    "pt_scene_num_triangles": (C.c_int, [C.c_void_p]),
    "pt_scene_build_bvh": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "pt_scene_num_nodes": (C.c_int, [C.c_void_p]),
    "pt_scene_depth": (C.c_int, [C.c_void_p]),
    "pt_scene_encode": (C.c_int, [C.c_void_p, c_float_p, c_float_p]),
    "pt_transform_matrix": (None, [c_float_p, c_float_p, c_float_p, c_float_p]),
    "pt_orbit_camera": (None, [C.c_float, C.c_float, C.c_float, c_float_p, c_float_p]),
    "pt_hdr_load": (C.c_int, [C.c_char_p, c_int_p, c_int_p, C.POINTER(c_float_p)]),
    "pt_hdr_decode": (C.c_int, [C.c_void_p, C.c_int64, c_int_p, c_int_p, C.POINTER(c_float_p)]),
    "pt_free": (None, [C.c_void_p]),
    "pt_hdr_cache": (C.c_int, [c_float_p, C.c_int, C.c_int, c_float_p]),
    "pt_hdr_cache_device": (C.c_int, [C.c_void_p, c_float_p, C.c_int, C.c_int, c_float_p]),
    "pt_image_write_pfm": (C.c_int, [C.c_char_p, c_float_p, C.c_int, C.c_int, C.c_int]),
    "pt_image_write_png": (C.c_int, [C.c_char_p, c_float_p, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int]),
}


_variant = None


def use_variant(name: str | None) -> None:
    """Select an in-tree tuning build (``_build.build_variant(name, ...)``) before the first
    load; used by tools/tune.py for A/B measurements. Names are restricted to [A-Za-z0-9_]."""
    import re
    global _variant
    if _lib is not None:
        raise RuntimeError("use_variant() must be called before the library is loaded")
    if name is not None and not re.fullmatch(r"[A-Za-z0-9_]{1,32}", name):
        raise ValueError(f"bad variant name {name!r}")
    _variant = name


def lib_path() -> Path:
    return _build.variant_lib(_variant) if _variant else _build.LIB


def _share_torch_hip_runtime():
    """One HIP runtime per process. PyTorch-ROCm bundles its own libamdhip64
    (its libraries ask for "libamdhip64.so", which does not match the
    "libamdhip64.so.7" soname libpt.so asks for), so loading libpt.so before
    torch puts two HIP/HSA runtimes in the process and whichever initialises
    second can fail to see the GPU. Importing torch first makes libpt.so bind to
    the already-loaded runtime (same soname). Without torch, libpt.so uses
    /opt/rocm's runtime."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(build_if_missing: bool = False):
    """Load libpt.so (raises if absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not path.exists():
        if not build_if_missing:
            raise RuntimeError(f"native library {path} is missing; run opengl_ray_tracing_amd._build.build_native()")
        _build.build_native()
    _share_torch_hip_runtime()
    lib = C.CDLL(str(path))
    lib.pt_abi_version.restype = C.c_int
    abi = lib.pt_abi_version()
    older_variant = _variant is not None and ABI_STRUCTS_SINCE <= abi < ABI_VERSION
    if abi != ABI_VERSION and not older_variant:  # the structs below must match the library's
        raise RuntimeError(f"{path} has ABI {abi}, this binding {ABI_VERSION}: rebuild it")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if older_variant:
                continue
            raise RuntimeError(f"{path} does not export {name}: rebuild it")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class PtError(RuntimeError):
    pass


def check(rc: int, ctx=None, what: str = ""):
    if rc != 0:
        msg = load().pt_last_error(ctx)
        raise PtError(f"{what} failed with {rc}: {msg.decode() if msg else ''}")
