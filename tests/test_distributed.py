"""Multi-rank screen-tile sharding on CPU (gloo, world_size 2 and 3): each rank
renders only its shard tiles (with the CPU restatement standing in for the
GPU kernel), packs them in the kernels' order, gathers to rank 0 and unpacks;
the reassembled frame must equal the single-rank frame bit for bit
(SURVEY.md 8(e))."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from opengl_ray_tracing_amd import distributed as D

W, H, SHARD = 200, 120, 32


def test_ownership_partitions_the_frame():
    for world in (1, 2, 3, 8):
        seen = np.zeros((H, W), np.int32)
        for r in range(world):
            p = D.owned_pixels(W, H, r, world, SHARD)
            seen[p[:, 1], p[:, 0]] += 1
            assert D.packed_count(W, H, r, world, SHARD) >= len(p)
        assert np.all(seen == 1)


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    a = rng.random((H, W, 4)).astype(np.float32)
    b = np.zeros_like(a)
    for r in range(3):
        D.unpack(b, D.pack(a, r, 3, SHARD), r, 3, SHARD)
    assert np.array_equal(a, b)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import torch

    import oracle
    from opengl_ray_tracing_amd import orbit_camera, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = scenes.scene_c2()
        s.build_bvh("sah", 8)
        tris, nodes = s.encode()
        env = scenes.synthetic_env(64, 32)
        eye, rot = orbit_camera(0, 0, 4)
        o = oracle.Oracle(tris, nodes, env)
        acc = np.zeros((H, W, 4), np.float32)
        mine = D.owned_pixels(W, H, rank, world, SHARD)
        for f in range(2):
            acc, _ = o.render(W, H, "lambert", f, eye, rot, accum=acc, pixels=mine, threads=1)
        maxc = max(D.packed_count(W, H, r, world, SHARD) for r in range(world))
        send = np.zeros((maxc, 4), np.float32)
        p = D.pack(acc, rank, world, SHARD)
        send[:len(p)] = p
        gl = [torch.zeros((maxc, 4)) for _ in range(world)] if rank == 0 else None
        dist.gather(torch.from_numpy(send), gather_list=gl, dst=0)
        if rank == 0:
            full = np.zeros((H, W, 4), np.float32)
            for r in range(world):
                n = D.packed_count(W, H, r, world, SHARD)
                D.unpack(full, gl[r].numpy()[:n], r, world, SHARD)
            ref = np.zeros((H, W, 4), np.float32)
            for f in range(2):
                ref, _ = o.render(W, H, "lambert", f, eye, rot, accum=ref, threads=1)
            q.put(bool(np.array_equal(full, ref)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_is_bit_exact(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def _sample_worker(rank, world, port, q):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    import torch

    import oracle
    from opengl_ray_tracing_amd import orbit_camera, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = scenes.scene_c2()
        s.build_bvh("sah", 8)
        tris, nodes = s.encode()
        env = scenes.synthetic_env(64, 32)
        eye, rot = orbit_camera(0, 0, 4)
        o = oracle.Oracle(tris, nodes, env)
        frames = 2
        acc = np.zeros((H, W, 4), np.float32)
        for f in range(frames):  # this rank's samples: f * world + rank
            acc, _ = o.render(W, H, "lambert", f, eye, rot, accum=acc, threads=1, sample_rank=rank,
                              sample_world=world)
        img = D.combine_sample_means(torch.from_numpy(acc.copy()), rank, world)
        if rank == 0:
            ref = np.zeros((H, W, 4), np.float32)
            for f in range(frames * world):  # one rank, samples 0 .. frames*world-1
                ref, _ = o.render(W, H, "lambert", f, eye, rot, accum=ref, threads=1)
            got = img.numpy()
            q.put(bool(np.allclose(got, ref, rtol=2e-5, atol=1e-6)) and bool(np.any(got != acc)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sample_parallel_mean(world):
    """Sample-parallel ranks (interleaved sample streams, one reduce when the image is consumed)
    give the single-rank running mean over the same samples, up to float summation order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sample_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def _bcast_worker(rank, world, port, q):
    from opengl_ray_tracing_amd import scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def build():
            s = scenes.scene_c2()
            s.build_bvh("sah", 8)
            tris, nodes = s.encode()
            return tris, nodes, scenes.synthetic_env(64, 32)

        tris, nodes, hdr = D.broadcast_scene(build, rank)
        tris2, nodes2, none = D.broadcast_scene(lambda: (np.arange(72.0), np.ones(12), None), rank)
        if rank != 0:  # every rank compares its arrays with a local build of the same scene
            rt, rn, rh = build()
            q.put(bool(np.array_equal(tris, rt) and np.array_equal(nodes, rn) and np.array_equal(hdr, rh)
                       and tris.dtype == np.float32 and np.array_equal(tris2, np.arange(72.0))
                       and nodes2.shape == (12,) and none is None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_broadcast_scene(world):
    """The scene built on rank 0 arrives bit-identical on every other rank (hdr may be None)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert all(q.get(timeout=5) is True for _ in range(world - 1))
