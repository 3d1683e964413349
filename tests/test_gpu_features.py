"""GPU feature tests through the C ABI: shared transcendentals (device == host
bits), the BASIC_CPU_COMPAT integrator, screen-tile sharding with on-device
pack/unpack, tonemap, error paths."""
import ctypes as C

import numpy as np
import pytest

import oracle
import parity
from opengl_ray_tracing_amd import Renderer, _native, orbit_camera, scenes
from opengl_ray_tracing_amd import distributed as D

pytestmark = pytest.mark.gpu
FP = C.POINTER(C.c_float)


def fmath(fn, x, y, ctx=None):
    lib = _native.load()
    out = np.empty_like(x)
    yp = None if y is None else y.ctypes.data_as(FP)
    if ctx is None:
        rc = lib.pt_fmath_host(fn, x.ctypes.data_as(FP), yp, x.size, out.ctypes.data_as(FP))
    else:
        rc = lib.pt_fmath_device(ctx, fn, x.ctypes.data_as(FP), yp, x.size, out.ctypes.data_as(FP))
    assert rc == 0
    return out


@pytest.mark.parametrize("fn", range(7))
def test_fmath_device_equals_host(fn):
    rng = np.random.default_rng(fn)
    n = 1 << 18
    if fn in (0, 1, 2):
        x = rng.uniform(-10, 10, n).astype(np.float32)
    elif fn == 3:
        x = rng.uniform(-1, 1, n).astype(np.float32)
    elif fn == 4:
        x = np.exp(rng.uniform(-80, 80, n)).astype(np.float32)
    elif fn == 5:
        x = rng.uniform(-90, 90, n).astype(np.float32)
    else:
        x = rng.uniform(1e-7, 1.0, n).astype(np.float32)
    y = rng.uniform(-3, 3, n).astype(np.float32) if fn in (2, 6) else None
    with Renderer(8, 8) as r:
        d = fmath(fn, x, y, r._h)
    h = fmath(fn, x, y)
    assert np.array_equal(d.view(np.uint32), h.view(np.uint32))


def test_basic_integrator_matches_oracle():
    """Counter-RNG mode: the double image and its f32 copy bit for bit against the oracle,
    which shares its arithmetic with the reference-pinned serial mode (test_basic_ref)."""
    sh = scenes.cornell_shapes()
    w = h = 256
    with Renderer(w, h, "basic", basic_samples=4) as r:
        r.upload_shapes(sh)
        for k in range(4):
            r.render_frame(np.zeros(3, np.float32), np.eye(4, dtype=np.float32), k)
        g = r.accum()
        gimg = r.basic_image()
        st = r.stats()
    o = oracle.Oracle(shapes=sh)
    acc = np.zeros((h, w, 4), np.float32)
    rays = 0
    for k in range(4):
        acc, c = o.render(w, h, "basic", k, accum=acc, basic_samples=4)
        rays += c.rays
    s = parity.assert_parity(g.reshape(-1, 4), acc.reshape(-1, 4), "basic")
    print("basic", s, "image bit-exact", np.array_equal(gimg, o.basic_image))
    assert np.array_equal(gimg.view(np.uint64), o.basic_image.view(np.uint64))
    assert np.array_equal(g.view(np.uint32), acc.view(np.uint32))
    assert int(st.rays) == rays


def test_basic_replay_equals_reference_image():
    """The GPU kernel replaying the reference's random stream (std::mt19937 seeded 5489, the
    draws of each pixel sample located by a serial pass of the checker) renders the reference
    CPU tracer's own image: its double image bit for bit (sha256 of tests/golden/basic/ref_s4,
    made by BasicRayTracingWithC++/main.cpp compiled from source) and its 8-bit output."""
    import hashlib
    import json
    from pathlib import Path

    from opengl_ray_tracing_amd.scene import imshow_bytes
    ref = json.loads((Path(__file__).resolve().parent / "golden" / "basic" / "ref_s4.json").read_text())
    sh = scenes.cornell_shapes()
    o = oracle.Oracle(shapes=sh)
    _, off, draws, c = o.basic_serial(samples=4, seed=ref["seed"], offsets=True)  # where each sample's draws start
    stream = oracle.mt_doubles(ref["seed"], draws)
    with Renderer(256, 256, "basic", basic_samples=4) as r:
        r.upload_shapes(sh)
        r.set_basic_stream(stream, off)
        for k in range(4):
            r.render_frame(np.zeros(3, np.float32), np.eye(4, dtype=np.float32), k)
        img = r.basic_image()
        over = r.basic_replay_overruns()
        st = r.stats()
    assert over == 0
    got = img.reshape(-1, 3)[ref["sample_index"]]
    print("replay: sampled pixels equal", np.array_equal(got, np.asarray(ref["sample_values"])))
    assert hashlib.sha256(img.tobytes()).hexdigest() == ref["image_f64_sha256"]
    assert hashlib.sha256(imshow_bytes(img).tobytes()).hexdigest() == ref["image_u8_sha256"]
    assert int(st.rays) == c.rays == 914124


def test_basic_checkpoint_restore_continues_the_image():
    """BASIC checkpoints: frames 0..4, the double image downloaded (pt_download_basic_image) and
    restored into a fresh context (pt_upload_basic_image), frames 5..9 there -- the double image
    and the f32 sums equal ten uninterrupted frames bit for bit. A restore from the f32 sums
    (pt_upload_accum, the generic checkpoint) sets the double image the next frame adds to: the
    sums widened."""
    sh = scenes.cornell_shapes()
    w, h = 96, 80
    z, eye4 = np.zeros(3, np.float32), np.eye(4, dtype=np.float32)

    def ctx():
        r = Renderer(w, h, "basic", basic_samples=10)
        r.upload_shapes(sh)
        return r

    with ctx() as r:
        for k in range(10):
            r.render_frame(z, eye4, k, sync=False)
        full_img, full_acc = r.basic_image(), r.accum()
    with ctx() as r:
        for k in range(5):
            r.render_frame(z, eye4, k, sync=False)
        img5, acc5 = r.basic_image(), r.accum()
    with ctx() as r:
        r.set_basic_image(img5)
        assert np.array_equal(r.accum()[..., :3], img5.astype(np.float32))
        for k in range(5, 10):
            r.render_frame(z, eye4, k, sync=False)
        assert np.array_equal(r.basic_image().view(np.uint64), full_img.view(np.uint64))
        assert np.array_equal(r.accum().view(np.uint32), full_acc.view(np.uint32))
    with ctx() as r:
        r.set_accum(acc5)
        assert np.array_equal(r.basic_image(), acc5[..., :3].astype(np.float64))
        r.render_frame(z, eye4, 5)
        assert not np.array_equal(r.accum(), acc5)  # the frame added to the restored sums


@pytest.mark.parametrize("world", [2, 4])
def test_tile_shards_reassemble_bit_exact(world):
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    w, h = 640, 360
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(w, h, "lambert") as full:
        full.upload_scene(tris, nodes)
        full.upload_env(hdr)
        for f in range(2):
            full.render_frame(eye, rot, f)
        ref = full.accum()
        total_rays = full.stats().rays
    ranks = [Renderer(w, h, "lambert", tile_rank=k, tile_world=world) for k in range(world)]
    rays = 0
    import torch  # device buffers for the packed shards (the RCCL path uses the same calls)
    for k, r in enumerate(ranks):
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(2):
            r.render_frame(eye, rot, f)
        rays += r.stats().rays
    # each rank touched exactly its own pixels
    for k, r in enumerate(ranks):
        a = r.accum()
        own = D.owned_pixels(w, h, k, world)
        mask = np.zeros((h, w), bool)
        mask[own[:, 1], own[:, 0]] = True
        assert np.all(a[~mask] == 0)
        assert np.array_equal(a[mask], ref[mask])
    # pack on each rank, unpack into rank 0 (what FrameGather does around dist.gather)
    bufs = []
    for k, r in enumerate(ranks):
        n = r.owned_pixel_count()
        assert n == D.packed_count(w, h, k, world)
        t = torch.zeros((n, 3), dtype=torch.float32, device="cuda:0")  # packed slots: r, g, b
        torch.cuda.synchronize()  # the fill runs on torch's stream, the pack on the renderer's
        r.pack_owned(t.data_ptr())
        r.synchronize()
        assert np.array_equal(t.cpu().numpy(), D.pack(ref, k, world)[:, :3])
        bufs.append(t)
    rank0 = ranks[0].accum()
    for k in range(1, world):
        ranks[0].unpack_rank(k, world, bufs[k].data_ptr())
    assert np.array_equal(ranks[0].accum(), ref)
    # the same reassembly in one launch (pt_unpack_ranks, FrameGather's accum mode)
    ranks[0].set_accum(rank0)
    ranks[0].unpack_ranks(world, [0] + [b.data_ptr() for b in bufs[1:]])
    assert np.array_equal(ranks[0].accum(), ref)
    assert rays == total_rays
    for r in ranks:
        r.close()


def test_tonemap_matches_pass3():
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(320, 180, "lambert") as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        r.render_frame(eye, rot, 0)
        a = r.accum()
        t = r.tonemap(1.5)
        tg = r.tonemap(1.5, 2.2)
    c = a[..., :3].astype(np.float32)
    lum = np.float32(0.3) * c[..., 0] + np.float32(0.6) * c[..., 1] + np.float32(0.1) * c[..., 2]
    want = c * (np.float32(1) / (np.float32(1) + lum / np.float32(1.5)))[..., None]
    assert np.allclose(t, want, rtol=1e-6, atol=1e-7)
    assert np.allclose(tg, np.power(want, 1 / 2.2), rtol=1e-5, atol=1e-6)


def _unorm8(x):
    """round(clamp(x, 0, 1) * 255) as the display kernels compute it: one fused multiply-add
    (exact in f64, then one rounding to f32), truncated."""
    c = np.clip(np.nan_to_num(x.astype(np.float32), nan=0.0), 0, 1).astype(np.float64)
    return np.floor((c * 255.0 + 0.5).astype(np.float32)).astype(np.uint8)


@pytest.mark.parametrize("gamma", [0.0, 2.2])
def test_display_frame_is_pass3_in_an_8bit_window(gamma):
    """pt_display_own of an unsplit context: every pixel's pass3 tonemap (the GPU's own f32
    tonemap, pt_tonemap) stored as an 8-bit unsigned-normalised RGBA pixel, alpha 255."""
    import torch
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(320, 180, "lambert") as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(2):
            r.render_frame(eye, rot, f)
        t = r.tonemap(1.5, gamma)
        img = torch.zeros((180, 320, 4), dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()  # the fill (torch's stream) before the renderer's stream writes it
        r.display_own(img.data_ptr(), 1.5, gamma)
        r.synchronize()
    got = img.cpu().numpy()
    assert np.array_equal(got[..., :3], _unorm8(t)) and np.all(got[..., 3] == 255)


def test_display_split_reassembles_the_frame():
    """Three tile ranks on one device: each packs its display pixels (3 u8 per owned slot), rank 0
    writes its own tiles and unpacks the other two in one launch -- the same RGBA8 frame as an
    unsplit context; rank 0's own tiles alone leave the others' pixels untouched."""
    import torch
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    W, H, world = 200, 130, 3
    full = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()  # torch's fills before the renderers' streams write these buffers
    with Renderer(W, H, "lambert") as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        r.render_frame(eye, rot, 0)
        r.display_own(full.data_ptr())
        r.synchronize()
    rs = [Renderer(W, H, "lambert", tile_rank=k, tile_world=world) for k in range(world)]
    try:
        packed = []
        for k, rr in enumerate(rs):
            rr.upload_scene(tris, nodes)
            rr.upload_env(hdr)
            rr.render_frame(eye, rot, 0)
            buf = torch.zeros(rr.owned_pixel_count() * 3, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            rr.display_pack(buf.data_ptr())
            rr.synchronize()
            packed.append(buf)
        img = torch.full((H, W, 4), 7, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        rs[0].display_own(img.data_ptr())
        rs[0].synchronize()
        own_only = img.cpu().numpy()
        rs[0].display_unpack(world, [0] + [b.data_ptr() for b in packed[1:]], img.data_ptr())
        rs[0].synchronize()
    finally:
        for rr in rs:
            rr.close()
    want = full.cpu().numpy()
    assert np.array_equal(img.cpu().numpy(), want)
    mine = np.zeros((H, W), bool)
    p = D.owned_pixels(W, H, 0, world)
    mine[p[:, 1], p[:, 0]] = True
    assert np.array_equal(own_only[mine], want[mine]) and np.all(own_only[~mine] == 7)


def test_error_paths():
    with Renderer(16, 16) as r:
        with pytest.raises(_native.PtError):
            r.render_frame(np.zeros(3, np.float32), np.eye(4, dtype=np.float32), 0)  # no scene
        bad = np.zeros((2, 12), np.float32)
        bad[1, 3], bad[1, 4] = 4, 10  # leaf range past the triangle array
        with pytest.raises(_native.PtError):
            r.upload_scene(np.zeros((3, 36), np.float32), bad)
    with pytest.raises(_native.PtError):
        Renderer(16, 16, device=99)


def caterpillar(n):
    """Encoded scene whose tree is a chain of depth n: node(l..r) = (node(l..r-1), leaf(r)).
    A ray along +x sees the nearer child internal at every level, so the traversal stack
    grows to n - 1 entries (beyond the LDS part, into the HBM overflow)."""
    tris = np.zeros((n, 36), np.float32)
    for i in range(n):
        x = float(i)
        tris[i, 0:9] = [x, 0, 0, x, 1, 0, x, 0, 1]
        tris[i, 9:18] = [1, 0, 0] * 3
        tris[i, 21:24] = [1, 1, 1]
    nodes = [np.array([255, 128, 0, 30, 0, 0, 1, 1, 0, 0, 1, 0], np.float32)]

    def box(l, r):
        p = tris[l:r + 1, 0:9].reshape(-1, 3)
        return p.min(0), p.max(0)

    def leaf(i):
        a, b = box(i, i)
        nodes.append(np.concatenate([[0, 0, 0, 1, i, 0], a, b]).astype(np.float32))
        return len(nodes) - 1

    def build(l, r):
        if l == r:
            return leaf(l)
        k = len(nodes)
        nodes.append(None)
        L = build(l, r - 1)
        R = leaf(r)
        a, b = box(l, r)
        nodes[k] = np.concatenate([[L, R, 0, 0, 0, 0], a, b]).astype(np.float32)
        return k

    assert build(0, n - 1) == 1
    return tris, np.stack(nodes)


@pytest.mark.parametrize("flags", [0, 1])
def test_deep_tree_uses_overflow_stack(flags):
    import sys
    sys.setrecursionlimit(10000)
    n = 200
    tris, nodes = caterpillar(n)
    rng = np.random.default_rng(3)
    m = 4000
    o = np.stack([np.full(m, -1.0), rng.uniform(0.05, 0.45, m), rng.uniform(0.05, 0.45, m)], 1)
    d = np.stack([np.ones(m), rng.normal(0, 0.05, m), rng.normal(0, 0.05, m)], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], 1).astype(np.float32)
    with Renderer(8, 8, flags=flags) as r:
        r.upload_scene(tris, nodes)
        t, tri = r.trace_closest(rays)
        assert r.stats().max_stack == n + 1
    t_o, tri_o, _ = oracle.Oracle(tris, nodes).trace_closest(rays)
    assert (tri_o == 0).mean() > 0.9
    assert np.array_equal(tri, tri_o) and np.array_equal(t, t_o)


def test_sample_parallel_streams():
    """Sample-parallel contexts (pt_config.sample_rank/sample_world) draw interleaved sample
    streams: their mean equals one context's running mean over the same samples (float order
    aside), and each stream is bit-exact against the CPU restatement."""
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    w, h, frames, world = 320, 180, 2, 2
    with Renderer(w, h, "lambert") as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(frames * world):
            r.render_frame(eye, rot, f)
        full = r.accum()
    parts = []
    for k in range(world):
        with Renderer(w, h, "lambert", sample_rank=k, sample_world=world) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for f in range(frames):
                r.render_frame(eye, rot, f)
            parts.append(r.accum())
    mean = (parts[0] + parts[1]) * np.float32(0.5)
    assert np.allclose(mean, full, rtol=2e-5, atol=1e-6)
    o = oracle.Oracle(tris, nodes, hdr)
    acc = np.zeros((h, w, 4), np.float32)
    for f in range(frames):
        acc, _ = o.render(w, h, "lambert", f, eye, rot, accum=acc, sample_rank=1, sample_world=world)
    assert np.array_equal(parts[1], acc)


@pytest.mark.parametrize("name", ["peppermint_powerplant_4k.hdr", "san_giuseppe_bridge_blurred.hdr"])
def test_hdr_cache_on_gpu_equals_host(name):
    """calculateHdrCache on the GPU (pt_envcache.hip) == the host restatement, bit for bit."""
    from pathlib import Path

    from opengl_ray_tracing_amd import calculate_hdr_cache, load_hdr
    import time
    hdr = load_hdr(Path(__file__).parent / "golden" / name)
    t0 = time.perf_counter()
    host = calculate_hdr_cache(hdr)
    t1 = time.perf_counter()
    with Renderer(8, 8) as r:
        r.hdr_cache_device(hdr)  # warm
        t2 = time.perf_counter()
        dev = r.hdr_cache_device(hdr)
        t3 = time.perf_counter()
    assert np.array_equal(dev.view(np.uint32), host.view(np.uint32))
    # the one sequential float sum bounds the device path (pt_envcache.hip hdrSumKernel)
    print(f"{name} {hdr.shape[1]}x{hdr.shape[0]}: host {1e3 * (t1 - t0):.1f} ms, device (incl. copies) "
          f"{1e3 * (t3 - t2):.1f} ms")


def test_launch_timing_ring_keeps_stats_exact():
    """Launch times live in a fixed ring of event pairs: rendering more frames than
    the ring holds keeps launches, the last frame's time and the summed time exact, and
    pt_reset_stats starts the totals over."""
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    eye, rot = orbit_camera(*cfg.camera)
    frames = 150  # > the 64-entry ring
    with Renderer(64, 36, "lambert") as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        per = []
        for f in range(frames):
            r.render_frame(eye, rot, f)
            st = r.stats()
            assert st.launches == f + 1
            per.append(st.kernel_ms)
        st = r.stats()
        assert st.launches == frames
        assert all(ms > 0 for ms in per)
        assert abs(st.kernel_ms_total - sum(per)) <= 1e-3 * sum(per)
        r.reset_stats()
        st = r.stats()
        assert st.launches == 0 and st.kernel_ms_total == 0.0 and st.rays == 0
        for f in range(frames):  # asynchronous frames: the ring back-pressures, nothing is lost
            r.render_frame(eye, rot, frames + f, sync=False)
        st = r.stats()
        assert st.launches == frames and st.kernel_ms_total > 0
        assert st.rays >= frames * 64 * 36


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_device_group_equals_one_device(devices):
    """One context over several devices (pt_config.n_devices; on the one-GPU box the same
    device repeated, so the gather runs as peer copies): every device renders its screen
    tiles and each frame gathers them into the first device's accumulation. The image equals
    a one-device render bit for bit across frames and a camera reset, with the same rays."""
    cfg, tris, nodes, hdr = scenes.build_config("c2")
    w, h = 480, 270
    eye, rot = orbit_camera(*cfg.camera)
    eye2, rot2 = orbit_camera(20.0, 10.0, 4.0)
    cams = [(eye, rot, f) for f in range(3)] + [(eye2, rot2, f) for f in range(2)]  # reset at frame 3

    def run(**kw):
        with Renderer(w, h, "lambert", **kw) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            imgs = []
            for e, m, f in cams:
                r.render_frame(e, m, f, sync=False)
                if f == 2:
                    imgs.append(r.accum())
            imgs.append(r.accum())
            return imgs, r.tonemap(1.5), r.stats()

    ref, ref_tm, ref_st = run()
    got, got_tm, st = run(devices=devices)
    assert st.devices == len(devices) and st.gather == 1  # PT_GATHER_COPY: the ids repeat
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    assert np.array_equal(got_tm, ref_tm)
    assert st.rays == ref_st.rays
    with pytest.raises(_native.PtError):  # RCCL needs distinct devices
        Renderer(w, h, "lambert", devices=devices, gather="rccl")


@pytest.mark.parametrize("name", ["c2", "c4"])
def test_camera_restart_keeps_policies_and_restarts_the_mean(name):
    """A camera move restarts the running mean (frameCounter 0, OpenglRayTracing/main.cpp:611-634):
    the next frames equal a fresh context's frames of the moved camera bit for bit, while the
    tree / split policies probed after the upload are kept (pt_runtime.cpp probePolicy)."""
    cfg, tris, nodes, hdr = scenes.build_config(name)
    w, h = 480, 270
    a = orbit_camera(*cfg.camera)
    b = orbit_camera(cfg.camera[0] + 7.0, cfg.camera[1] + 3.0, cfg.camera[2])
    with Renderer(w, h, cfg.integrator, max_bounce=cfg.max_bounce) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(24):  # past the 20-frame policy probe
            r.render_frame(*a, f)
        tree = r.stats().runtime_tree
        for f in range(3):
            r.render_frame(*b, f)
        moved = r.accum()
        assert r.stats().runtime_tree == tree
    with Renderer(w, h, cfg.integrator, max_bounce=cfg.max_bounce) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(3):
            r.render_frame(*b, f)
        fresh = r.accum()
    assert np.array_equal(moved, fresh)


@pytest.mark.parametrize("name", ["c2", "c4"])
def test_band_order_frames_equal_ordered_frames(name):
    """Frames handed out in band order (PT_FLAG_NO_TILE_ORDER) give the longest-first frames' image bit for bit,
    across the probe and a camera restart (the megakernel's tile hand-out: FLAG_MEGAKERNEL, as
    Lambert frames default to the regen kernel)."""
    from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_NO_TILE_ORDER
    cfg, tris, nodes, hdr = scenes.build_config(name)
    w, h = 480, 270
    a = orbit_camera(*cfg.camera)
    b = orbit_camera(cfg.camera[0] + 7.0, cfg.camera[1] + 3.0, cfg.camera[2])

    def run(flags):
        with Renderer(w, h, cfg.integrator, max_bounce=cfg.max_bounce, flags=flags | FLAG_MEGAKERNEL) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for f in range(24):
                r.render_frame(*a, f, sync=False)
            first = r.accum()
            for f in range(4):
                r.render_frame(*b, f, sync=False)
            return first, r.accum(), r.stats().rays

    x, y = run(0), run(FLAG_NO_TILE_ORDER)
    assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1])
    assert x[2] == y[2]


def test_compact_env_texels_for_radiance_maps_only():
    """A Radiance map's texels (RGBE values) and calculateHdrCache's table (float(x) / w) are read
    from their compact form (8 + 4 bytes per texel instead of 16 + 8), which decodes to the uploaded
    floats bit for bit, and the table by rows (env_compact 2: a row record and the distinct rows'
    2-byte y's, pt_kernels.h Env::cacheRow; the megakernel's MIS light samples read it, here the
    4-bounce frames); an env that does not
    round-trip -- the synthetic sky of the smoke test -- keeps the float texels, and all give the
    oracle's image (the parity tests render with the compact forms too)."""
    cfg, tris, nodes, hdr = scenes.build_config("c4")  # san_giuseppe: the megakernel reads its table by rows
    eye, rot = orbit_camera(*cfg.camera)
    w, h = 96, 54
    for integ, mb in (("lambert", 2), ("mis", 2), ("mis", 4)):
        for name, env in [("radiance", hdr), ("synthetic", scenes.synthetic_env(128, 64))]:
            with Renderer(w, h, integ, max_bounce=mb) as r:
                r.upload_scene(tris, nodes)
                r.upload_env(env)
                r.render_frame(eye, rot, 0)
                st = r.stats()
                assert st.env_compact == (2 if name == "radiance" else 0), name
                g = r.accum()
            o, _ = oracle.Oracle(tris, nodes, env).render(w, h, integ, 0, eye, rot, max_bounce=mb)
            parity.assert_parity(g.reshape(-1, 4), o.reshape(-1, 4), f"env/{integ}{mb}/{name}")
