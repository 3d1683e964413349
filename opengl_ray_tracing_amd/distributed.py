"""Multi-GPU rendering, one process per GPU. Two ways to split
the per-pixel path:

* screen tiles (strong scaling): tiles of `shard` x `shard` pixels dealt
  round-robin over the ranks (tile t belongs to rank t % world); one gather of
  the packed shards to rank 0 per presented frame over RCCL/xGMI (FrameGather).
  Every pixel's value depends only on (pixel, frameCounter) and its own running
  mean (pass1.fsh:73-76, :118-122, :868-871), so the reassembled frame is
  bit-identical to a single-GPU render. The packed order (tile, row, column)
  matches the kernels in csrc/pt_kernels.hip (packKernel / unpackKernel).
* sample streams (weak scaling): every rank renders the whole frame from its
  own interleaved sample stream (pt_config.sample_rank / sample_world: rank r
  draws samples r, r+W, r+2W, ...), with no collective per frame; the image is
  the mean of the ranks' running means, combined by one RCCL reduce when it is
  consumed (SampleReduce). Equal to the single-GPU mean over the same samples up
  to float summation order.
"""
from __future__ import annotations

import numpy as np


def shard_grid(width: int, height: int, shard: int = 32):
    return (width + shard - 1) // shard, (height + shard - 1) // shard


def owned_tiles(width: int, height: int, rank: int, world: int, shard: int = 32) -> np.ndarray:
    sx, sy = shard_grid(width, height, shard)
    return np.arange(rank, sx * sy, world, dtype=np.int64)


def packed_count(width: int, height: int, rank: int, world: int, shard: int = 32) -> int:
    return int(owned_tiles(width, height, rank, world, shard).size) * shard * shard


def packed_coords(width: int, height: int, rank: int, world: int, shard: int = 32):
    """(px, py, valid) of every packed slot, in the kernels' (tile, row, col) order."""
    sx, _ = shard_grid(width, height, shard)
    g = owned_tiles(width, height, rank, world, shard)
    within = np.arange(shard * shard, dtype=np.int64)
    gy, gx = (g // sx)[:, None], (g % sx)[:, None]
    px = (gx * shard + within[None] % shard).ravel()
    py = (gy * shard + within[None] // shard).ravel()
    valid = (px < width) & (py < height)
    return px, py, valid


def owned_pixels(width: int, height: int, rank: int, world: int, shard: int = 32) -> np.ndarray:
    px, py, v = packed_coords(width, height, rank, world, shard)
    return np.stack([px[v], py[v]], 1).astype(np.int32)


def pack(accum: np.ndarray, rank: int, world: int, shard: int = 32) -> np.ndarray:
    h, w = accum.shape[:2]
    px, py, v = packed_coords(w, h, rank, world, shard)
    out = np.zeros((px.size, accum.shape[2]), accum.dtype)
    out[v] = accum[py[v], px[v]]
    return out


def unpack(accum: np.ndarray, packed: np.ndarray, rank: int, world: int, shard: int = 32) -> None:
    h, w = accum.shape[:2]
    px, py, v = packed_coords(w, h, rank, world, shard)
    accum[py[v], px[v]] = packed[v]


class FrameGather:
    """RCCL gather of every rank's screen-tile shard to rank 0, once per frame.

    Two things to gather (`mode`):

    * "display" -- the frame as presented (pass3.fsh tonemap into the reference's 8-bit
      GLUT_RGBA window, ImportanceSampling_LowDiscrepancySequence/main.cpp:706,747): every
      rank packs its tiles' display values (3 bytes per pixel, pt_display_pack), rank 0
      writes its own tiles and unpacks the others' into an H x W x 4 u8 image
      (pt_display_own / pt_display_unpack). A quarter of the accumulation's bytes cross
      xGMI per frame; each rank's running mean stays with it (`gather_accum()` brings the
      whole accumulation to rank 0 when it is wanted, bit-identical to a 1-GPU render).
    * "accum" -- the running mean itself (3 f32 per pixel, pt_pack_owned / pt_unpack_ranks: the
      other ranks' buffers in one launch) into rank 0's accumulation after every batch of frames.

    Device buffers are torch tensors (torch is the allocator/collective plumbing here).
    The renderer runs on a torch stream of its own; each call packs the frame just
    rendered into one of two send buffers and runs the gather -- and on rank 0 the
    unpack -- on a communication stream, so frame f's gather overlaps frame f+1's render
    (rank 0's render writes only its own tiles, the unpack only the others'). A send
    buffer (and, in display mode, an image) is written again only after its previous
    gather finished. `synchronize()` completes the last frame's gather. `overlap=False`
    runs everything on the render stream.
    """

    def __init__(self, renderer, rank: int, world: int, device, overlap: bool = True, mode: str = "accum",
                 limit: float = 1.5, gamma: float = 0.0, proxy: bool = False):
        """proxy: one process on one GPU times rank `rank`'s share of the split with its real
        per-batch work -- the pack, and on rank 0 the unpack of every other rank's buffer -- but
        no collective (the receive buffers keep what they hold; tools/shard_time.py)."""
        import torch
        import torch.distributed as dist

        if mode not in ("accum", "display"):
            raise ValueError(f"mode {mode!r}")
        self.torch, self.dist = torch, dist
        self.proxy = proxy
        self.r, self.rank, self.world, self.device = renderer, rank, world, device
        self.mode, self.limit, self.gamma = mode, float(limit), float(gamma)
        counts = [renderer.owned_pixel_count(k, world) for k in range(world)]
        self.maxc = max(counts)
        self.overlap = overlap and (proxy or not _staged())
        # the renderer gets a stream of its own that torch knows about (torch's default
        # stream has the handle 0, which pt_set_stream reads as "the context's own stream")
        self.render_stream = torch.cuda.Stream(device)
        self.comm_stream = torch.cuda.Stream(device) if self.overlap else self.render_stream
        nbuf = 2 if self.overlap else 1
        if mode == "display":  # packed slots: 3 u8 (r, g, b of the displayed pixel)
            shape, dtype = (self.maxc * 3,), torch.uint8
        else:  # packed slots: 3 f32 (r, g, b; pt_pack_owned), 12 bytes per pixel over xGMI
            shape, dtype = (self.maxc, 3), torch.float32
        self.send = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(nbuf)]
        self.recv = [torch.zeros(shape, dtype=dtype, device=device) for _ in range(world)] \
            if rank == 0 else None
        self.images = [torch.zeros((renderer.height, renderer.width, 4), dtype=torch.uint8, device=device)
                       for _ in range(nbuf)] if (mode == "display" and rank == 0) else None
        self._recv_ptrs = [0] + [t.data_ptr() for t in self.recv[1:]] if self.recv is not None else None
        self.packed = [torch.cuda.Event() for _ in range(nbuf)]
        self.done = [torch.cuda.Event() for _ in range(nbuf)]
        self.used = [False] * nbuf  # the buffer's done event has been recorded
        self.k = 0
        self.last = None  # index of the image holding the last presented frame (rank 0, display mode)
        torch.cuda.current_stream(device).synchronize()  # the buffers' fills, before the other streams use them
        renderer.set_stream(self.render_stream.cuda_stream)

    @property
    def image(self):
        """Rank 0, display mode: the last presented frame (H x W x 4 u8, device), complete
        once its gather has (synchronize(), or the comm stream's done event)."""
        return None if self.images is None or self.last is None else self.images[self.last]

    def _pack(self, i):
        if self.mode == "display":
            if self.rank == 0:
                self.r.display_own(self.images[i].data_ptr(), self.limit, self.gamma)
            else:
                self.r.display_pack(self.send[i].data_ptr(), self.limit, self.gamma)
        else:
            self.r.pack_owned(self.send[i].data_ptr())

    def _unpack(self, i):
        if self.mode == "display":
            self.r.display_unpack(self.world, self._recv_ptrs, self.images[i].data_ptr())
        else:  # every other rank's running means in one launch (pt_unpack_ranks)
            self.r.unpack_ranks(self.world, self._recv_ptrs)

    def __call__(self):
        torch, dist = self.torch, self.dist
        i = self.k % len(self.send)
        self.k += 1
        if self.used[i]:
            self.render_stream.wait_event(self.done[i])
        self._pack(i)  # on the render stream, after the frame
        if self.mode == "display" and self.rank == 0:
            self.last = i
        if not self.proxy and _staged():  # gloo rehearsal: the collective on host copies, ordered after the pack
            with torch.cuda.stream(self.render_stream):
                host = self.send[i].cpu()
                recv = [torch.zeros_like(host) for _ in range(self.world)] if self.rank == 0 else None
                dist.gather(host, gather_list=recv, dst=0)
                if self.rank == 0:
                    for t, h in zip(self.recv, recv):
                        t.copy_(h)
                    self._unpack(i)
            return
        self.packed[i].record(self.render_stream)
        with torch.cuda.stream(self.comm_stream):
            self.comm_stream.wait_event(self.packed[i])
            if not self.proxy:
                dist.gather(self.send[i], gather_list=self.recv, dst=0)
            if self.rank == 0:
                self.r.set_stream(self.comm_stream.cuda_stream)
                self._unpack(i)
                self.r.set_stream(self.render_stream.cuda_stream)
            self.done[i].record(self.comm_stream)
        self.used[i] = True

    def gather_accum(self):
        """Bring every rank's running mean to rank 0's accumulation (3 f32 per pixel, once,
        synchronous): rank 0 then holds the whole accumulation, bit-identical to a 1-GPU
        render. Collective: every rank calls it."""
        torch, dist = self.torch, self.dist
        self.synchronize()
        with torch.cuda.stream(self.render_stream):  # every allocation, copy and kernel in one stream order
            buf = torch.zeros((self.maxc, 3), dtype=torch.float32, device=self.device)
            self.r.pack_owned(buf.data_ptr())
            recv = [torch.zeros_like(buf) for _ in range(self.world)] if self.rank == 0 else None
            if _staged():
                host = buf.cpu()
                hrecv = [torch.zeros_like(host) for _ in range(self.world)] if self.rank == 0 else None
                dist.gather(host, gather_list=hrecv, dst=0)
                if self.rank == 0:
                    for t, h in zip(recv, hrecv):
                        t.copy_(h)
            else:
                dist.gather(buf, gather_list=recv, dst=0)
            if self.rank == 0:
                self.r.unpack_ranks(self.world, [0] + [t.data_ptr() for t in recv[1:]])
        self.render_stream.synchronize()

    def synchronize(self):
        self.comm_stream.synchronize()
        self.render_stream.synchronize()


def _staged() -> bool:
    """True when the process group is gloo (CPU rehearsal of the RCCL path): device tensors
    are staged through host copies around the collective."""
    import torch.distributed as dist

    return dist.get_backend() == "gloo"


def combine_sample_means(img, rank: int, world: int):
    """Mean over ranks of equally weighted running means (in place on rank 0's `img`)."""
    import torch.distributed as dist

    if img.is_cuda and _staged():
        h = img.cpu()
        dist.reduce(h, dst=0, op=dist.ReduceOp.SUM)
        img.copy_(h)
    else:
        dist.reduce(img, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        img.mul_(1.0 / world)
    return img


class SampleReduce:
    """RCCL reduce of every rank's running mean (sample-parallel rendering) to rank 0.

    The renderer's accumulation is copied (device to device, on the renderer's
    stream = torch's current stream) into a torch buffer which is summed to rank
    0 and scaled by 1/world; the ranks' own running means are left untouched.
    """

    def __init__(self, renderer, rank: int, world: int, device):
        import torch

        self.r, self.rank, self.world = renderer, rank, world
        self.torch = torch
        self.img = torch.empty((renderer.height, renderer.width, 4), dtype=torch.float32, device=device)
        self.stream = torch.cuda.Stream(device)
        renderer.set_stream(self.stream.cuda_stream)

    def __call__(self):
        self.r.accum_into(self.img.data_ptr())  # synchronous on the renderer's stream
        with self.torch.cuda.stream(self.stream):
            return combine_sample_means(self.img, self.rank, self.world)


def broadcast_scene(build, rank: int, device=None):
    """Build the scene once on rank 0 and broadcast it to every rank.

    The reference uploads its TBOs once from the one process it has
    (OpenglRayTracing/main.cpp:720-735); with one process per GPU every rank
    needs the same arrays, and running the host BVH build on all ranks at once
    only makes them contend for the host cores. `build()` -> (tris, nodes, hdr)
    runs on rank 0 alone; the arrays then travel as one broadcast each (device
    tensors over RCCL/xGMI, host tensors under gloo) and come back as host
    numpy arrays ready for Renderer.upload_scene / upload_env. Returns
    (tris, nodes, hdr) on every rank, bit-identical to rank 0's; hdr may be None.
    """
    import torch
    import torch.distributed as dist

    arrays = build() if rank == 0 else (None, None, None)
    shapes = [None if a is None else tuple(np.asarray(a).shape) for a in arrays]
    obj = [shapes]
    dist.broadcast_object_list(obj, src=0)
    shapes = obj[0]
    on_device = device is not None and not _staged()
    out = []
    for a, shp in zip(arrays, shapes):
        if shp is None:
            out.append(None)
            continue
        if rank == 0:
            a = np.ascontiguousarray(a, np.float32)
            t = torch.from_numpy(a)
        else:
            t = torch.empty(shp, dtype=torch.float32)
        if on_device:
            t = t.to(device)
        dist.broadcast(t, src=0)
        out.append(a if rank == 0 else t.cpu().numpy())
    return tuple(out)
