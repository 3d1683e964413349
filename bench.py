#!/usr/bin/env python3
"""Benchmark: Mrays/s and ms/frame at 1 spp per frame (BASELINE.json metric).

A step is one progressive frame (one display() of OpenglRayTracing/main.cpp:558-603)
of the configured workload on every rank: 1 spp for every pixel of the frame,
running-mean accumulate. Default workload: configs[1] = c2, the
OpenglRayTracing bunny scene (5k tris) at 1920x1080, Lambert, 2 bounces.

N > 1 ranks (one process per GPU):
  --shard tiles (default, strong scaling: BASELINE north_star's split): every
      rank renders its 32x32 screen tiles of the one frame, in batches of frames per
      launch (pt_render_frames_async: each frame 1 spp and its own running-mean update;
      the renderer's batchFor: 12 x N for Lambert at the box's 4 hardware queues, at
      most 32);
      after every batch the running means of the rank's pixels (f32 radiance,
      12 B/pixel) are gathered to rank 0 over RCCL (bit-exact reassembly),
      pipelined one batch deep: batch b's gather runs on a communication stream
      while batch b+1 renders. --gather display moves the displayed frame
      (pass3 tonemap in the 8-bit window, 3 B/pixel) instead.
  --shard samples (weak scaling): every rank renders the whole frame from its
      own interleaved sample stream (rank r: samples r, r+N, ...), no
      collective per step; the ranks' running means are combined by one RCCL
      reduce after the timed steps (validated, not timed).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver launch for N > 1)

Rank 0 prints one JSON line (contract in the task statement), with
``roofline`` for a frame: the work the hardware counters measured for every kernel
of a frame (camera-ray pass, frame kernel, tile reorder, running-mean update: VALU
wave-instructions, DRAM-side bytes; committed under profiles/<round>/counters.json by
tools/roofline.py) over this run's live wall time per frame (and, as kernel_basis,
over the serially issued frames' HIP-event time), against each resource's peak --
``bound`` is the resource with the
highest fraction -- plus ``equivalent_GBs``, the reference algorithm's fetch
bytes per launch over the same duration; and ``cpu_baseline``
(the CPU restatement of the reference on the host cores, rank 0 at N = 1); and ``per_call``
(N = 1): the median wall time of 100 synchronous pt_render_frame calls after 10 warm-up calls,
SURVEY 8(d)'s ms/frame -- one display() per call, what INTEGRATION.md's drop-in gets.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# hardware queues for the renderer's frames in flight (one stream each, pt_runtime.cpp depthStep):
# the package's one policy (opengl_ray_tracing_amd/__init__.py, also what the tests run under) --
# 12 when GPU_MAX_HW_QUEUES is unset, an explicit value respected (at most 32) -- applied at import,
# before torch or the renderer first initialises HIP; the line reports the value in effect
import opengl_ray_tracing_amd  # noqa: E402,F401

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue: 1024 SIMD-32s (256 CUs x 4) each issue one wave64 VALU instruction per 2 cycles
# at the 2.4 GHz maximum clock (MI355X_MICROARCH.md "Wave scheduling"): 1228.8 G wave-instructions/s
VALU_PEAK_GINST = 1024 * 2.4 / 2 * 1e9 / 1e9
METRIC = "Mrays/sec + ms/frame (1 spp, 1080p) at 1/2/4/8 MI355X; CPU-ref spp-matched PSNR"
PROBE_FRAMES = 90  # frames after a restart during which the renderer measures its policies (tree, split, order, depth)
SERIAL_FRAMES = 20  # frames of the serial-frames run behind roofline.kernel_basis
PER_CALLS, PER_CALL_WARMUP = 100, 10  # per_call: SURVEY 8(d)'s median of 100 pt_render_frame calls after 10


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--builder", default=None, help="override the config's BVH builder")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true", help="skip the spp-matched PSNR check")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="cpu_baseline sample: full frames are rendered until this much CPU wall time has passed")
    ap.add_argument("--counters", default=str(ROOT / "profiles" / "r6" / "counters.json"),
                    help="per-launch PMC counters of the bench kernel per config (tools/roofline.py)")
    ap.add_argument("--no-reset", action="store_true", help="skip the reset_ms_per_frame frames (profiling runs)")
    ap.add_argument("--no-serial", action="store_true", help="skip the serial-frames run (roofline.kernel_basis)")
    ap.add_argument("--no-per-call", action="store_true", help="skip the per_call run (profiling runs)")
    ap.add_argument("--cpu-all-seconds", type=float, default=4.0,
                    help="cpu_baseline.all_cores sample: full frames at nproc threads for this long (0: skip)")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL); gloo only to rehearse N > 1 on one GPU")
    ap.add_argument("--same-device", action="store_true", help="rehearsal: every rank on device 0")
    ap.add_argument("--gather", choices=["display", "accum"], default="accum",
                    help="--shard tiles: after every batch of frames, gather the running means (f32 radiance, "
                         "3 f32 per pixel) or the displayed frame (RGB8, 3 B/pixel; the running means then "
                         "gathered once after the run)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch (pt_config.frame_batch; 0 = the renderer's choice: 2 x tile_world, "
                         "tile_world on large Disney/MIS scenes)")
    ap.add_argument("--shard", choices=["samples", "tiles"], default="tiles",
                    help="N > 1: sample-parallel full frames (weak) or screen-tile shards of one frame (strong)")
    return ap.parse_args()


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def main():
    args = parse()
    rank, world, local = dist_env()
    if world != args.gpus and world > 1:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    n = world

    if os.environ.get("PT_VARIANT"):  # A/B of an in-tree tuning build (tools/tune.py --build); not a default run
        from opengl_ray_tracing_amd import _native
        _native.use_variant(os.environ["PT_VARIANT"])
    from opengl_ray_tracing_amd import FLAG_COUNT_FETCHES, Renderer, orbit_camera, scenes

    torch = None
    if n > 1:
        import torch
        import torch.distributed as dist
        if args.same_device:
            local = 0
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend, init_method="env://")
        # the scene is prepared once, on rank 0, and broadcast: N ranks building c5's
        # 1M-triangle tree at once would only contend for the host's cores
        from opengl_ray_tracing_amd.distributed import broadcast_scene
        cfg = scenes.CONFIGS[args.config]
        if cfg.integrator == "basic":  # the BASIC shapes are 19 records of doubles: built locally
            cfg, tris, nodes, hdr = scenes.build_config(args.config, args.builder)
        else:
            tris, nodes, hdr = broadcast_scene(lambda: scenes.build_config(args.config, args.builder)[1:], rank,
                                               None if args.dist_backend == "gloo" else f"cuda:{local}")
    else:
        cfg, tris, nodes, hdr = scenes.build_config(args.config, args.builder)
    eye, rot = orbit_camera(*cfg.camera)

    tiles = n > 1 and args.shard == "tiles"
    split = dict(tile_rank=rank, tile_world=n) if tiles else dict(sample_rank=rank, sample_world=n)
    r = Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, device=local,
                 flags=args.flags, frame_batch=args.batch, **split)
    r.upload_scene(tris, nodes)
    r.upload_env(hdr)

    # ---- algorithmic bytes per ray of the reference algorithm, counted on the GPU by the
    # instrumented kernel variant (no culling, closest-hit shadows: exactly pass1.fsh's fetches)
    rc = Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, device=local,
                  flags=FLAG_COUNT_FETCHES, **split)
    rc.upload_scene(tris, nodes)
    rc.upload_env(hdr)
    rc.render_frame(eye, rot, 0)
    cs = rc.stats()
    rc.close()
    bytes_per_ray = (48 * cs.node_fetch + 72 * cs.tri_fetch + 72 * cs.mat_fetch + 12 * cs.tex_fetch) / max(cs.rays, 1)

    # ---- multi-GPU: RCCL gather of every rank's screen-tile shard to rank 0;
    # the renderer runs on torch's current stream so the collective orders after the frame
    gather = combine = None
    if tiles:
        from opengl_ray_tracing_amd.distributed import FrameGather
        gather = FrameGather(r, rank, n, f"cuda:{local}", mode=args.gather)
    elif n > 1:
        from opengl_ray_tracing_amd.distributed import SampleReduce
        combine = SampleReduce(r, rank, n, f"cuda:{local}")

    batch = r.stats().frame_batch  # frames per launch = frames per gather (the renderer's: 2 x N for Lambert)

    def frames(first, n, cam=None, per=None):
        """frames first .. first+n-1: batches of `per` (default `batch`) frames (one launch each, every
        frame its own 1 spp and running-mean update), each followed by the gather to rank 0 when N > 1"""
        e, c = cam if cam is not None else (eye, rot)
        per = per or batch
        k = 0
        while k < n:
            m = min(per, n - k)
            r.render_frames(e, c, first + k, m)
            if gather is not None:
                gather()
            k += m

    def sync_all():
        r.synchronize()
        if n > 1:
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    # The renderer picks its tree and tile-split policies from measurements on the
    # first 13 frames after a running-mean restart (pt_runtime.cpp probePolicy); those
    # frames run before the W warmup steps, so the timed frames are the
    # progressive steady state (same image, bit for bit, either way).
    frames(0, PROBE_FRAMES)
    frames(PROBE_FRAMES, args.warmup)
    sync_all()
    r.reset_stats()
    t0 = time.perf_counter()
    frames(PROBE_FRAMES + args.warmup, args.steps)
    sync_all()
    t1 = time.perf_counter()
    st = r.stats()
    # N > 1: the same steps with one gather per frame (one frame per launch), the cadence at which
    # the reference presents (IS main.cpp:706), timed the same way -- reported next to the batched
    # figure, whose image reaches rank 0 once per batch of `batch` frames
    per_frame_ms = per_frame_rays = None
    if gather is not None and batch > 1:
        sync_all()
        r.reset_stats()
        t4 = time.perf_counter()
        frames(PROBE_FRAMES + args.warmup + args.steps, args.steps, per=1)
        sync_all()
        per_frame_ms = 1e3 * (time.perf_counter() - t4) / args.steps
        per_frame_rays = r.stats().rays  # this window's own rays (other sample indices than the batched window's)
    # what the reference's caller gets per display() (ms/frame = the wall time of one
    # pt_render_frame, median of 100 frames after 10 warm-up frames; INTEGRATION.md binds one call per
    # display(), OpenglRayTracing/main.cpp:558-603): synchronous single-frame calls continuing the
    # same running mean, each timed on the host around the call (its ctypes crossing included)
    per_call = None
    if n == 1 and PER_CALLS > 0 and not args.no_per_call:
        f0 = PROBE_FRAMES + args.warmup + args.steps
        for k in range(PER_CALL_WARMUP):
            r.render_frame(eye, rot, f0 + k)
        r.reset_stats()
        ts = []
        for k in range(PER_CALLS):
            ta = time.perf_counter()
            r.render_frame(eye, rot, f0 + PER_CALL_WARMUP + k)
            ts.append(1e3 * (time.perf_counter() - ta))
        sp = r.stats()
        ts.sort()
        med = float(np.median(ts))
        rpf = sp.rays / max(sp.frames, 1)
        per_call = {"ms_median": round(med, 4), "ms_p10": round(ts[len(ts) // 10], 4),
                    "ms_p90": round(ts[(9 * len(ts)) // 10], 4), "value": round(rpf / (med * 1e-3) / 1e6, 2),
                    "unit": "Mrays/s", "calls": PER_CALLS, "warmup_calls": PER_CALL_WARMUP,
                    "kernel_ms": round(sp.kernel_ms_total / max(sp.launches, 1), 4),
                    "what": "one synchronous pt_render_frame per display(), frames issued one at a time"}
    # interactive cost after a camera move (the reference's mouse() rotates the camera and zeroes
    # frameCounter, OpenglRayTracing/main.cpp:611-634): frames 0..PROBE_FRAMES-1 of a restarted
    # running mean from a camera rotated by one degree, timed like the steps -- the camera-ray
    # bins are rebuilt and the per-tile split state starts over; the tree / split policies
    # probed after the upload are kept (pt_runtime.cpp probePolicy)
    reset_ms = None
    if not args.no_reset:
        moved = orbit_camera(cfg.camera[0] + 1.0, *cfg.camera[1:])
        t2 = time.perf_counter()
        frames(0, PROBE_FRAMES, moved)
        sync_all()
        reset_ms = 1e3 * (time.perf_counter() - t2) / PROBE_FRAMES
    # the frame kernel's own duration with nothing overlapping it: the same workload with frames
    # issued serially (PT_FLAG_SERIAL_FRAMES, full-residency grid), HIP events around each launch.
    # With frames in flight a launch's duration spans the frames it overlaps, so the roofline's
    # second basis (kernel_basis) divides the same per-launch work by this serial duration.
    serial_ms = None
    if rank == 0 and n == 1 and not args.no_serial:
        from opengl_ray_tracing_amd import FLAG_SERIAL_FRAMES
        with Renderer(cfg.width, cfg.height, cfg.integrator, max_bounce=cfg.max_bounce, device=local,
                      flags=args.flags | FLAG_SERIAL_FRAMES) as rs:
            rs.upload_scene(tris, nodes)
            rs.upload_env(hdr)
            for f in range(PROBE_FRAMES):
                rs.render_frame(eye, rot, f, sync=False)
            rs.synchronize()
            rs.reset_stats()
            for f in range(SERIAL_FRAMES):
                rs.render_frame(eye, rot, PROBE_FRAMES + f, sync=False)
            rs.synchronize()
            ss = rs.stats()
            serial_ms = ss.kernel_ms_total / max(ss.launches, 1)
    combined_finite = combined_filled = None
    if gather is not None:  # rank 0's accumulation: every rank's running means (not timed)
        if args.gather == "display":  # the running means to rank 0, once
            gather.gather_accum()
        gather.synchronize()
        r.synchronize()
        if rank == 0:
            a = r.accum()
            combined_finite = bool(np.isfinite(a).all())
            combined_filled = round(float((a[..., 3] == 1.0).mean()), 4)  # every pixel mixed (alpha 1) at least once
    if combine is not None:  # the ranks' running means -> one image on rank 0 (after the timed steps)
        img = combine()
        torch.cuda.synchronize()
        combined_finite = bool(torch.isfinite(img).all().item()) if rank == 0 else None

    elapsed = t1 - t0
    rays_local = st.rays
    if n > 1:
        dev = "cpu" if args.dist_backend == "gloo" else f"cuda:{local}"
        tt = torch.tensor([elapsed, float(rays_local), st.kernel_ms_total], dtype=torch.float64, device=dev)
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item())
        if reset_ms is not None:
            rs = torch.tensor([reset_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(rs, op=dist.ReduceOp.MAX)
            reset_ms = float(rs[0].item())
        if per_frame_ms is not None:
            pf = torch.tensor([per_frame_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(pf, op=dist.ReduceOp.MAX)
            per_frame_ms = float(pf[0].item())
            pr = torch.tensor([float(per_frame_rays)], dtype=torch.float64, device=dev)
            dist.all_reduce(pr, op=dist.ReduceOp.SUM)
            per_frame_rays = float(pr[0].item())
        rays_total = float(sm[1].item())
        kernel_ms_avg = float(mx[2].item()) / max(st.launches, 1)
    else:
        rays_total = float(rays_local)
        kernel_ms_avg = st.kernel_ms_total / max(st.launches, 1)

    if rank == 0:
        ms_per_step = 1e3 * elapsed / args.steps
        mrays = rays_total / elapsed / 1e6
        rays_per_frame = rays_local / max(st.frames, 1)
        # frames in flight overlap their kernels, so a launch's own duration overstates its share of
        # the device: the roofline then divides by the wall time per frame (frame kernel + reorder +
        # running-mean update) instead
        pipelined = st.frames_in_flight > 1
        roofline = make_roofline(args, cfg, ms_per_step if pipelined else kernel_ms_avg, rays_per_frame,
                                 bytes_per_ray, n, "frame")
        roofline["time_basis"] = ("wall ms per frame (frames in flight)" if pipelined
                                  else "frame kernel HIP-event ms")
        roofline["launch_ms"] = round(kernel_ms_avg, 4)
        roofline["kernel"] = ("regenKernel<%s>" if st.regen else "renderKernel<%s>") % cfg.integrator
        if serial_ms is not None:
            kb = make_roofline(args, cfg, serial_ms, rays_per_frame, bytes_per_ray, n, "frame_serial")
            roofline["kernel_basis"] = {
                "time_basis": "frame kernel HIP-event ms, frames issued serially (PT_FLAG_SERIAL_FRAMES)",
                "kernel_ms": round(serial_ms, 4), "frames": SERIAL_FRAMES, "bound": kb["bound"],
                "frac": kb["frac"], "candidates": kb.get("candidates"), "equivalent_GBs": kb["equivalent_GBs"]}
        cpu = None
        if not args.no_cpu_baseline and n == 1:
            cpu = cpu_baseline(cfg, tris, nodes, hdr, eye, rot, args.cpu_seconds, args.cpu_all_seconds)
        quality = spp_matched_psnr(local) if not args.no_psnr else None
        line = {
            "metric": METRIC, "value": round(mrays, 2), "unit": "Mrays/s", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "probe_frames": PROBE_FRAMES, "ms_per_step": round(ms_per_step, 4),
            "reset_ms_per_frame": None if reset_ms is None else round(reset_ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.shard == "tiles" else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{cfg.name}: {cfg.description}", "resolution": f"{cfg.width}x{cfg.height}",
                       "spp_per_frame": 1, "integrator": cfg.integrator, "max_bounce": cfg.max_bounce,
                       "triangles": int(tris.shape[0]), "bvh_nodes": int(nodes.shape[0]),
                       "bvh_builder": args.builder or cfg.builder, "env": cfg.env,
                       # the tree the timed frames traversed: the uploaded one, or the runtime's own
                       # binned-SAH tree with every result checked against the uploaded one
                       "traversal_tree": "runtime (checked against uploaded)" if st.runtime_tree else "uploaded",
                       "frame_kernel": "path regeneration" if st.regen else "lock-step megakernel",
                       "waves_per_simd": st.waves_per_simd, "frames_in_flight": st.frames_in_flight,
                       "hw_queues": opengl_ray_tracing_amd.HW_QUEUES,
                       "frames_per_launch": batch, "frames_per_gather": batch if n > 1 else None,
                       "parallelism": (f"screen-tile x{n}" + ((f" + RCCL gather of the displayed frame (RGB8) per "
                                                               f"batch of {batch} frames" if args.gather == "display"
                                                               else f" + RCCL gather of the running means (f32 "
                                                               f"radiance) per batch of {batch} frames")
                                                              if n > 1 else ""))
                       if args.shard == "tiles" else
                       (f"sample-parallel x{n}" + (" (RCCL reduce of the running means after the run)"
                                                   if n > 1 else ""))},
            "roofline": roofline, "cpu_baseline": cpu, "quality": quality,
        }
        if combined_finite is not None:
            line["config"]["combined_image_finite"] = combined_finite
        if combined_filled is not None:
            line["config"]["combined_image_filled"] = combined_filled
        if per_call is not None:
            line["per_call"] = per_call
        if per_frame_ms is not None:  # the same frames with a gather after every frame
            line["gather_every_frame"] = {"ms_per_step": round(per_frame_ms, 4),
                                          "value": round(per_frame_rays / (per_frame_ms * 1e-3 * args.steps) / 1e6, 2),
                                          "unit": "Mrays/s", "frames_per_gather": 1}
        print(json.dumps(line), flush=True)
    r.close()
    if n > 1:
        dist.destroy_process_group()


def make_roofline(args, cfg, kernel_ms, rays_per_frame, bytes_per_ray, n, basis="frame"):
    """Roofline of a frame. Each resource's work per frame comes from the hardware counters of the
    same workload (profiles/<round>/counters.json, tools/roofline.py, one rocprofv3 pass per counter
    group over this bench's timed frames), summed over every kernel of the frame (basis "frame":
    camera-ray pass, frame kernel, tile reorder, running-mean update -- over the wall time per
    frame) or over the kernels of a serially issued frame ("frame_serial": no running-mean update
    kernel -- over their summed HIP-event time); divided by this run's live time it gives the
    achieved rate:
      valu: SQ_INSTS_VALU wave-instructions / t  vs 1228.8 G/s (1024 SIMDs x 2.4 GHz / 2 cycles)
      hbm:  (2*FETCH_SIZE + WRITE_SIZE) KiB / t  vs 8 TB/s (gfx950 FETCH_SIZE halving corrected)
    `bound` is the resource with the higher fraction. `equivalent_GBs` is the reference
    algorithm's fetch bytes (48 F_node + 72 F_tri + 72 F_mat + 12 F_tex per ray,
    counted by the instrumented kernel) over the same time -- what pass1.fsh would have to
    move, not what this kernel moves (its tree, culling and packets fetch far less)."""
    t = kernel_ms * 1e-3
    eq = rays_per_frame * bytes_per_ray / t / 1e9
    base = {"kernel": "renderKernel<%s>" % cfg.integrator, "kernel_ms": round(kernel_ms, 4),
            "equivalent_GBs": round(eq, 1), "bytes_per_ray": round(bytes_per_ray, 1),
            "rays_per_frame": int(rays_per_frame)}
    ent = None
    p = Path(args.counters) if args.counters else None
    if p and p.exists() and not args.flags and not args.builder and n == 1:
        ent = json.loads(p.read_text()).get(args.config)
    if not ent:
        return {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
                "note": "no committed counters for this workload", **base}
    work = ent.get(basis) or {"kernels": ["frame"], "valu_insts": ent["valu_insts"], "dram_bytes": ent["dram_bytes"]}
    cands = {
        "valu": (work["valu_insts"] / t / 1e9, VALU_PEAK_GINST, "G VALU wave-instructions/s"),
        "hbm": (work["dram_bytes"] / t / 1e9, HBM_PEAK_GBS, "GB/s"),
    }
    bound = max(cands, key=lambda k: cands[k][0] / cands[k][1])
    a, pk, unit = cands[bound]
    return {"bound": bound, "achieved": round(a, 2), "peak": pk, "unit": unit, "frac": round(a / pk, 4),
            "traffic": int(work["dram_bytes"]),
            "candidates": {k: {"achieved": round(v[0], 2), "peak": v[1], "unit": v[2], "frac": round(v[0] / v[1], 4)}
                           for k, v in cands.items()},
            "counters": {"source": str(p.relative_to(ROOT)) if p.is_relative_to(ROOT) else str(p),
                         "kernels": work["kernels"], "valu_insts_per_frame": work["valu_insts"],
                         "dram_bytes_per_frame": work["dram_bytes"],
                         "l2_hit": ent.get("l2_hit"), "profiled_kernel_ms": ent.get("kernel_ms")},
            **base}


def spp_matched_psnr(device: int, spp: int = 128):
    """The metric's "CPU-ref spp-matched PSNR": the BasicRayTracingWithC++ scene (config c1, 256x256)
    rendered by the GPU BASIC_CPU_COMPAT integrator at 128 spp, imshow'd (main.cpp:183) and
    compared with the reference's own 4000 spp image, beside what the reference CPU tracer itself
    scores at 128 spp (tests/golden/basic/ref_s128.json: that program compiled from its source,
    std::mt19937 seeded 5489)."""
    import json

    from PIL import Image

    from opengl_ray_tracing_amd import Renderer, scenes
    from opengl_ray_tracing_amd.scene import imshow_bytes
    gold = ROOT / "tests" / "golden" / "4000spp.png"
    fix = ROOT / "tests" / "golden" / "basic" / f"ref_s{spp}.json"
    if not gold.exists():
        return None
    with Renderer(256, 256, "basic", basic_samples=spp, device=device) as r:
        r.upload_shapes(scenes.cornell_shapes())
        z, eye4 = np.zeros(3, np.float32), np.eye(4, dtype=np.float32)
        t0 = time.perf_counter()
        for k in range(spp):
            r.render_frame(z, eye4, k, sync=False)
        r.synchronize()
        dt = time.perf_counter() - t0
        img = imshow_bytes(r.basic_image())
    ref = np.asarray(Image.open(gold))[..., :3].astype(np.float64)
    psnr = 10 * np.log10(255.0 ** 2 / np.mean((img.astype(np.float64) - ref) ** 2))
    ref_psnr = json.loads(fix.read_text())["psnr_vs_4000spp_db"] if fix.exists() else None
    return {"psnr_db": round(float(psnr), 2), "reference_psnr_db": None if ref_psnr is None else round(ref_psnr, 2),
            "reference_source": str(fix.relative_to(ROOT)), "spp": spp,
            "scene": "c1 BasicRayTracingWithC++ Cornell box 256x256", "vs": "4000spp.png (reference)",
            "render_ms": round(dt * 1e3, 2)}


def cpu_baseline(cfg, tris, nodes, hdr, eye, rot, seconds, all_seconds=0.0):
    """The CPU restatement of the reference (oracle/, test infrastructure) timed on the host
    cores: full frames of the same workload (same scene, camera, frame sequence), OpenMP over
    pixels, until `seconds` of wall time have passed (a bounded sample)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle  # noqa: E402  (bench.py's cpu_baseline leg is the only bench use of oracle/)

    host = host_cpu()
    cores = host["threads"]
    orc = oracle.Oracle(tris, nodes, hdr)

    def sample(threads, secs):
        acc = np.zeros((cfg.height, cfg.width, 4), np.float32)
        rays = frames = 0
        t0 = time.perf_counter()
        while True:
            acc, c = orc.render(cfg.width, cfg.height, cfg.integrator, frames, eye, rot, accum=acc,
                                max_bounce=cfg.max_bounce, threads=threads)
            rays += c.rays
            frames += 1
            if time.perf_counter() - t0 >= secs:
                break
        dt = time.perf_counter() - t0
        return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
                "sample": f"{frames} full {cfg.width}x{cfg.height} frames of {cfg.name} ({rays} rays, {dt:.1f} s)",
                "ms_per_frame": round(1e3 * dt / frames, 1)}

    out = {**sample(cores, seconds), "host": host}
    # the CPU tracer on all host cores of the box too (nproc threads, however many
    # of them the job's CPU share actually runs), beside the per-GPU share above
    if all_seconds > 0 and host["nproc"] > cores:
        out["all_cores"] = sample(host["nproc"], all_seconds)
    return out


def host_cpu():
    """The host cores the CPU baseline may use: every CPU in this process's affinity mask,
    bounded by the job's CPU share when the environment states one (OMP_NUM_THREADS: the GPU
    box grants 16 cores per GPU and says so there; nproc shows the whole machine)."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    share = os.environ.get("OMP_NUM_THREADS", "")
    threads = min(affinity, int(share)) if share.isdigit() and int(share) > 0 else affinity
    model = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None  # the job's CPU bandwidth limit (cgroup v2 cpu.max: quota/period CPUs), if any
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"threads": max(1, threads), "nproc": nproc, "affinity": affinity,
            "omp_num_threads": share or None, "cgroup_cpus": quota, "cpu_model": model}


if __name__ == "__main__":
    main()
