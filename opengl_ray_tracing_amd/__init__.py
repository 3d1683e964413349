"""MI355X-native progressive path tracer with the host surface of
xfause/OpenGL_Ray_Tracing (include/pt_abi.h).

Hot path: hand-written HIP kernels for gfx950 in csrc/, reached through the
C ABI of libpt.so. There is no CPU fallback in this package.

Frames in flight run on a HIP stream each. HIP reads GPU_MAX_HW_QUEUES
(hardware queues per process, its default 4) once, when it first initialises: importing this
package sets it to 12 only when it is unset and HIP is not initialised yet (an explicit value is
left alone), and records the value in effect (HW_QUEUES), which every Renderer passes to the
runtime as pt_config.hw_queues -- the pipeline is sized to the queues the process really has.
"""
import os
import sys


def _hip_initialised() -> bool:
    torch = sys.modules.get("torch")
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:  # noqa: BLE001  (a partial torch import)
        return False


def _hw_queues(want: int = 12) -> int:
    cur = os.environ.get("GPU_MAX_HW_QUEUES", "")
    if not cur and not _hip_initialised():
        os.environ["GPU_MAX_HW_QUEUES"] = cur = str(want)
    return min(int(cur), 32) if cur.isdigit() and int(cur) > 0 else 4


HW_QUEUES = _hw_queues()

from .scene import (Material, Scene, calculate_hdr_cache, decode_hdr, get_transform_matrix, load_hdr,
                    orbit_camera, read_pfm, write_pfm, write_png)
from .renderer import (FLAG_CLOSEST_SHADOW, FLAG_COUNT_FETCHES, FLAG_NO_CULL, FLAG_NO_TILE_ORDER, FLAG_REFERENCE_TREE, FLAG_SERIAL_FRAMES, FLAG_NO_BINS, FLAG_HOST_ACCEL, FLAG_MEGAKERNEL, FLAG_PRIMARY_PASS, FLAG_REGEN, FLAG_WAVEFRONT, INTEGRATORS,
                       FrameStats, Renderer, device_count)

__all__ = [
    "Material", "Scene", "calculate_hdr_cache", "decode_hdr", "get_transform_matrix", "load_hdr", "orbit_camera",
    "read_pfm", "write_pfm", "write_png",
    "Renderer", "FrameStats", "device_count", "INTEGRATORS", "FLAG_NO_CULL", "FLAG_CLOSEST_SHADOW",
    "FLAG_COUNT_FETCHES", "FLAG_HOST_ACCEL", "FLAG_MEGAKERNEL", "FLAG_PRIMARY_PASS", "FLAG_NO_TILE_ORDER", "FLAG_REFERENCE_TREE", "FLAG_REGEN", "FLAG_WAVEFRONT",
]
