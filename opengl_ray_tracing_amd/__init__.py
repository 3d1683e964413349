"""MI355X-native progressive path tracer with the host surface of
xfause/OpenGL_Ray_Tracing (include/pt_abi.h).

Hot path: hand-written HIP kernels for gfx950 in csrc/, reached through the
C ABI of libpt.so. There is no CPU fallback in this package.

Frames in flight run on a HIP stream each: importing the package raises
GPU_MAX_HW_QUEUES (hardware queues per process, HIP's default 4) to 12 unless
PT_KEEP_HW_QUEUES is set; HIP reads it once, when it first initialises, so import this
package before torch or anything else initialises HIP. The renderer sizes its pipeline
to the queues the variable grants.
"""
import os


def _hw_queues(want: int = 12) -> None:
    if os.environ.get("PT_KEEP_HW_QUEUES"):
        return
    cur = os.environ.get("GPU_MAX_HW_QUEUES", "")
    if not cur.isdigit() or int(cur) < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want)


_hw_queues()

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
