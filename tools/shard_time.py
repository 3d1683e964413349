#!/usr/bin/env python3
"""Per-rank frame time of the screen-tile split, measured on one GPU: rank 0's
share of an N-way split (its 32x32 tiles t % N == 0) rendered alone, wall ms per
frame with frames in flight and frames batched per launch (pt_render_frames_async,
PT_BATCH frames per launch, 0 = the renderer's choice; PT_BATCH_MUL = m: m x N). The N-GPU frame is at
least this plus whatever of the per-batch gather does not overlap the next batch.

    [PT_VARIANT=<tuning build>] [PT_BATCH=b | PT_BATCH_MUL=m] python tools/shard_time.py [config] [N ...]
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
# the bench's hardware queues (bench.py): 12, so the frames in flight get a queue each
import os  # noqa: E402
if not os.environ.get("GPU_MAX_HW_QUEUES", "").isdigit() or int(os.environ["GPU_MAX_HW_QUEUES"]) < 12:
    os.environ["GPU_MAX_HW_QUEUES"] = "12"

import opengl_ray_tracing_amd  # noqa: E402,F401


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    worlds = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
    import os

    import torch  # noqa: F401  (one HIP runtime with torch, as in bench.py)
    from opengl_ray_tracing_amd import _native
    if os.environ.get("PT_VARIANT"):  # an in-tree tuning build (tools/tune.py --build)
        _native.use_variant(os.environ["PT_VARIANT"])
    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    cfg, tris, nodes, hdr = scenes.build_config(cfg_name)
    eye, rot = orbit_camera(*cfg.camera)
    batch = int(os.environ.get("PT_BATCH", "0"))
    mul = int(os.environ.get("PT_BATCH_MUL", "0"))  # frames per launch = mul x N (overrides PT_BATCH)
    for n in worlds:
        with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, tile_rank=0,
                      tile_world=n, frame_batch=mul * n if mul else batch) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            r.render_frames(eye, rot, 0, 100)  # policy probe (tree, split, order) + warmup
            r.synchronize()
            r.reset_stats()
            K = int(os.environ.get("PT_SHARD_FRAMES", "200"))  # 20: the driver's bench line, from an idle GPU
            t0 = time.perf_counter()
            r.render_frames(eye, rot, 100, K)
            t_sub = time.perf_counter()
            r.synchronize()
            ms = 1e3 * (time.perf_counter() - t0) / K
            submit_ms = 1e3 * (t_sub - t0) / K  # host time per pt_render_frame_async call
            st = r.stats()
        print(json.dumps({"variant": os.environ.get("PT_VARIANT", "base"), "config": cfg_name, "world": n, "rank0_ms_per_frame": round(ms, 4),
                          "frames": st.frames, "launches": st.launches, "frame_batch": st.frame_batch,
                          "kernel_ms_avg": round(st.kernel_ms_total / max(st.launches, 1), 4),
                          "host_submit_ms": round(submit_ms, 4),
                          "rays_per_frame": st.rays // max(st.frames, 1),
                          "frames_in_flight": st.frames_in_flight}), flush=True)


if __name__ == "__main__":
    main()
