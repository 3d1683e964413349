"""Multi-process screen-tile rendering through the HIP path: spawned ranks each
drive a Renderer (libpt.so on the GPU) over their own 32x32 tiles and present
every frame on rank 0 with FrameGather. On the one-GPU box
every rank shares device 0 and the collective is gloo (staged through host
copies); the reassembled frame must equal a single-context render bit for bit.
A world-1 RCCL group drives FrameGather's overlapped path (gather and unpack
on the communication stream, double-buffered packs). In display mode the ranks
present each frame as 8-bit display pixels; the presented image must equal a
single-context display of the same frame, and gather_accum() the accumulation."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H, FRAMES = 320, 180, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _render_full(cfg, tris, nodes, hdr, eye, rot):
    import torch

    from opengl_ray_tracing_amd import Renderer
    with Renderer(W, H, cfg.integrator, max_bounce=cfg.max_bounce) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(FRAMES):
            r.render_frame(eye, rot, f)
        img = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()  # the fill (torch's stream) before the renderer's stream writes it
        r.display_own(img.data_ptr())
        r.synchronize()
        return r.accum(), r.stats().rays, img.cpu().numpy()


def _tile_worker(rank, world, port, backend, q, mode):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch
    import torch.distributed as dist

    from opengl_ray_tracing_amd import Renderer, orbit_camera, scenes
    from opengl_ray_tracing_amd.distributed import FrameGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        cfg, tris, nodes, hdr = scenes.build_config("c2")
        eye, rot = orbit_camera(*cfg.camera)
        r = Renderer(W, H, cfg.integrator, max_bounce=cfg.max_bounce, device=0, tile_rank=rank, tile_world=world)
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        g = FrameGather(r, rank, world, "cuda:0", mode=mode)
        for f in range(FRAMES):
            r.render_frame(eye, rot, f, sync=False)
            g()
        g.synchronize()
        torch.cuda.synchronize()
        rays = torch.tensor([float(r.stats().rays)], device="cpu" if backend == "gloo" else "cuda:0")
        dist.all_reduce(rays)
        shown = g.image.cpu().numpy() if (mode == "display" and rank == 0) else None
        if mode == "display":
            g.gather_accum()
        if rank == 0:
            got = r.accum()
            ref, ref_rays, ref_img = _render_full(cfg, tris, nodes, hdr, eye, rot)
            bad = np.argwhere(np.any(got != ref, axis=-1))
            if len(bad):
                from opengl_ray_tracing_amd import distributed as D
                own = np.zeros((H, W), np.int32) - 1
                for k in range(world):
                    p = D.owned_pixels(W, H, k, world)
                    own[p[:, 1], p[:, 0]] = k
                print("mismatch", len(bad), "owners", np.bincount(own[bad[:, 0], bad[:, 1]], minlength=world),
                      "got", got[bad[0][0], bad[0][1]], "ref", ref[bad[0][0], bad[0][1]], flush=True)
            exact = bool(np.array_equal(got, ref))
            if mode == "display":
                img_ok = bool(np.array_equal(shown, ref_img)) and bool(np.all(shown[..., 3] == 255))
                if not img_ok:
                    bad = np.argwhere(np.any(shown != ref_img, axis=-1))
                    print("display mismatch", len(bad), "first", bad[:3].tolist(), shown[tuple(bad[0])],
                          ref_img[tuple(bad[0])], flush=True)
                print("accum exact", exact, "image exact", img_ok, flush=True)
                exact = exact and img_ok
            q.put((exact, int(rays.item()) == ref_rays, g.overlap))
        r.close()
    finally:
        dist.destroy_process_group()


def _spawn(world, backend, mode="accum"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tile_worker, args=(r, world, port, backend, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return q.get(timeout=5)


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_render_tiles_and_gather_bit_exact(world):
    exact, rays_ok, overlap = _spawn(world, "gloo")
    assert exact and rays_ok and not overlap


def test_rccl_world1_overlapped_gather_path():
    """FrameGather with a real RCCL group (world 1 on the one-GPU box): the overlapped
    path -- pack on the render stream, gather + unpack on the communication stream, two
    send buffers -- leaves the frame exact."""
    exact, rays_ok, overlap = _spawn(1, "nccl")
    assert exact and rays_ok and overlap


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_present_display_frames_bit_exact(world):
    """Display mode: 3 bytes per pixel per frame to rank 0; the presented RGBA8 frame equals a
    single-context pt_display_own of the same frame, and gather_accum() the accumulation."""
    exact, rays_ok, overlap = _spawn(world, "gloo", "display")
    assert exact and rays_ok and not overlap


def test_rccl_world1_overlapped_display_path():
    exact, rays_ok, overlap = _spawn(1, "nccl", "display")
    assert exact and rays_ok and overlap
