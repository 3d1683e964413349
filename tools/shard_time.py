#!/usr/bin/env python3
"""Per-rank frame time of the screen-tile split, measured on one GPU: rank 0's
share of an N-way split (its 32x32 tiles t % N == 0) rendered alone, wall ms per
frame with frames in flight and frames batched per launch (pt_render_frames_async,
PT_BATCH frames per launch, 0 = the renderer's choice; PT_BATCH_MUL = m: m x N), issued
exactly as bench.py issues them -- batches of the renderer's frames per launch, each followed
by rank 0's real per-batch work (distributed.FrameGather(proxy=True): the pack of its own tiles
on the render stream, and the one-launch unpack of the other N - 1 ranks' buffers into its
accumulation on the communication stream) but no collective (PT_SHARD_GATHER=0: render only).
The N-GPU frame is this plus whatever of the xGMI gather itself does not overlap the next batch.

    [PT_VARIANT=<tuning build>] [PT_BATCH=b | PT_BATCH_MUL=m] [PT_SHARD_FRAMES=K] [PT_SHARD_FLAGS=f]
        python tools/shard_time.py [config] [N ...]
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
# hardware queues: the package's policy (opengl_ray_tracing_amd/__init__.py), as bench.py and the tests
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
    from opengl_ray_tracing_amd.distributed import FrameGather
    with_gather = os.environ.get("PT_SHARD_GATHER", "1") != "0"
    for n in worlds:
        with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, tile_rank=0,
                      tile_world=n, frame_batch=mul * n if mul else batch,
                      flags=int(os.environ.get("PT_SHARD_FLAGS", "0"), 0)) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            g = FrameGather(r, 0, n, "cuda:0", mode="accum", proxy=True,
                            overlap=os.environ.get("PT_SHARD_OVERLAP", "1") != "0") if with_gather and n > 1 else None
            per = r.stats().frame_batch

            def frames(first, k):  # bench.py's frames(): batches, each followed by the gather
                while k > 0:
                    m = min(per, k)
                    r.render_frames(eye, rot, first, m)
                    if g is not None:
                        g()
                    first += m
                    k -= m

            frames(0, 100)  # policy probe (tree, split, order) + warmup
            r.synchronize()
            if g is not None:
                g.synchronize()
            r.reset_stats()
            K = int(os.environ.get("PT_SHARD_FRAMES", "200"))  # 20: the driver's bench line, from an idle GPU
            if os.environ.get("SHARD_TRACE"):  # a PT_WAVE_TRACE build records the timed frames' waves only
                os.environ["PT_WAVE_TRACE_FILE"] = f"{os.environ['SHARD_TRACE']}_{cfg_name}_n{n}.bin"
            t0 = time.perf_counter()
            frames(100, K)
            t_sub = time.perf_counter()
            r.synchronize()
            if g is not None:
                g.synchronize()
            ms = 1e3 * (time.perf_counter() - t0) / K
            os.environ.pop("PT_WAVE_TRACE_FILE", None)
            submit_ms = 1e3 * (t_sub - t0) / K  # host time per pt_render_frame_async call
            st = r.stats()
        print(json.dumps({"variant": os.environ.get("PT_VARIANT", "base"), "config": cfg_name, "world": n, "rank0_ms_per_frame": round(ms, 4),
                          "frames": st.frames, "launches": st.launches, "frame_batch": st.frame_batch,
                          "kernel_ms_avg": round(st.kernel_ms_total / max(st.launches, 1), 4),
                          "host_submit_ms": round(submit_ms, 4),
                          "rays_per_frame": st.rays // max(st.frames, 1), "gather": g is not None,
                          "hw_queues": opengl_ray_tracing_amd.HW_QUEUES,
                          "frames_in_flight": st.frames_in_flight}), flush=True)


if __name__ == "__main__":
    main()
