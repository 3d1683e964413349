"""GPU parity: the HIP path (through the C ABI of libpt.so) against the CPU
restatement of the reference (oracle/pt_oracle.c) on the same seeded inputs.

Traversal/intersection results and rendered pixels are compared bit-exactly
(tests/parity.py asserts exact == 1.0 together with the stated tolerance bar and
linear PSNR >= 60 dB, which every failure message reports).
"""
import numpy as np
import pytest

import oracle
import parity
from opengl_ray_tracing_amd import FLAG_COUNT_FETCHES, FLAG_NO_CULL, Renderer, orbit_camera, scenes

pytestmark = pytest.mark.gpu

W, H = 1920, 1080


@pytest.fixture(scope="module")
def c2():
    return scenes.build_config("c2")


@pytest.fixture(scope="module")
def c3():
    return scenes.build_config("c3")


@pytest.fixture(scope="module")
def c4():
    return scenes.build_config("c4")


def random_rays(eye, n, seed):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(np.asarray(eye, np.float64)[None], n, 0) + 0.3 * rng.normal(size=(n, 3))
    return np.concatenate([o, d], 1).astype(np.float32)


@pytest.mark.parametrize("flags", [0, FLAG_NO_CULL, 0x40])  # 0x40 = FLAG_REFERENCE_TREE
def test_trace_closest_bit_exact(c2, flags):
    cfg, tris, nodes, hdr = c2
    orc = oracle.Oracle(tris, nodes)
    eye, _ = orbit_camera(0, 0, 4)
    rays = random_rays(eye, 20000, 1)
    with Renderer(64, 64, "lambert", flags=flags) as r:
        r.upload_scene(tris, nodes)
        t, tri = r.trace_closest(rays)
    t_o, tri_o, _ = orc.trace_closest(rays)
    assert (tri_o >= 0).mean() > 0.2
    assert np.array_equal(tri, tri_o)
    assert np.array_equal(t, t_o)


def test_trace_closest_exact_ties():
    """Every triangle twice, so every hit is an exact-t tie decided by the reference's
    visiting order: the runtime tree flags the ties and retraces those rays through the
    uploaded tree, giving the oracle's triangle for every ray."""
    from opengl_ray_tracing_amd import Material, Scene
    n = 24
    u, v = np.meshgrid(np.linspace(-1, 1, n), np.linspace(-1, 1, n))
    verts = np.stack([u.ravel(), 0.2 * np.sin(3 * u.ravel()) * np.cos(2 * v.ravel()), v.ravel()], 1)
    idx = []
    for i in range(n - 1):
        for j in range(n - 1):
            a = i * n + j
            idx += [[a, a + 1, a + n], [a + 1, a + n + 1, a + n]]
    idx = np.array(idx, np.int32)
    s = Scene()
    s.add_mesh(verts.astype(np.float32), idx, Material())
    s.add_mesh(verts.astype(np.float32), idx, Material())
    s.build_bvh("sah", 8)
    tris, nodes = s.encode()
    rng = np.random.default_rng(7)
    o = np.stack([rng.uniform(-0.8, 0.8, 20000), np.full(20000, 2.0), rng.uniform(-0.8, 0.8, 20000)], 1)
    d = np.stack([rng.normal(0, 0.2, 20000), -np.ones(20000), rng.normal(0, 0.2, 20000)], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], 1).astype(np.float32)
    with Renderer(64, 64, "lambert") as r:
        r.upload_scene(tris, nodes)
        t, tri = r.trace_closest(rays)
    t_o, tri_o, _ = oracle.Oracle(tris, nodes).trace_closest(rays)
    assert (tri_o >= 0).mean() > 0.2
    assert np.array_equal(tri, tri_o)
    assert np.array_equal(t, t_o)


def render_gpu(cfg, tris, nodes, hdr, frames=1, flags=0, integrator=None, max_bounce=None, w=W, h=H, stream=False):
    """frames synchronous display() calls (pt_render_frame), or stream=True: one asynchronous stream of
    frames (pt_render_frames_async, batched launches)"""
    eye, rot = orbit_camera(*cfg.camera)
    with Renderer(w, h, integrator or cfg.integrator, max_bounce=cfg.max_bounce if max_bounce is None else max_bounce,
                  flags=flags) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        if stream:
            r.render_frames(eye, rot, 0, frames)
        else:
            for f in range(frames):
                r.render_frame(eye, rot, f)
        return r.accum(), r.stats()


def render_oracle(cfg, tris, nodes, hdr, pixels, frames=1, integrator=None, max_bounce=None, w=W, h=H):
    eye, rot = orbit_camera(*cfg.camera)
    orc = oracle.Oracle(tris, nodes, hdr)
    acc = np.zeros((h, w, 4), np.float32)
    cnt = None
    for f in range(frames):
        acc, cnt = orc.render(w, h, integrator or cfg.integrator, f, eye, rot, accum=acc, pixels=pixels,
                              max_bounce=cfg.max_bounce if max_bounce is None else max_bounce)
    return acc, cnt


@pytest.mark.parametrize("name,integrator", [("c2", "lambert"), ("c3", "disney"), ("c3", "mis"), ("c4", "mis")])
def test_render_parity(request, name, integrator):
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    mb = {"disney": 5}.get(integrator, cfg.max_bounce)
    px = parity.sample_pixels(W, H, 20000, seed=7)
    g, st = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator=integrator, max_bounce=mb)
    o, _ = render_oracle(cfg, tris, nodes, hdr, px, frames=2, integrator=integrator, max_bounce=mb)
    gs, os_ = g[px[:, 1], px[:, 0]], o[px[:, 1], px[:, 0]]
    s = parity.assert_parity(gs, os_, f"{name}/{integrator}")
    print(name, integrator, s, "rays", st.rays)
    assert np.all(g[..., 3] == 1.0)


def test_cull_matches_reference_traversal(c2):
    cfg, tris, nodes, hdr = c2
    a, sa = render_gpu(cfg, tris, nodes, hdr, frames=1)
    b, sb = render_gpu(cfg, tris, nodes, hdr, frames=1, flags=FLAG_NO_CULL)
    assert sa.rays == sb.rays
    assert np.mean(np.all(a == b, axis=-1)) > 0.9999


def test_fetch_counts_match_oracle(c2):
    """FLAG_COUNT_FETCHES reproduces the reference algorithm's fetch counts (roofline bytes)."""
    cfg, tris, nodes, hdr = c2
    w, h = 480, 270
    g, st = render_gpu(cfg, tris, nodes, hdr, frames=1, flags=FLAG_COUNT_FETCHES, w=w, h=h)
    o, cnt = render_oracle(cfg, tris, nodes, hdr, None, frames=1, w=w, h=h)
    # per-pixel branch flips may move a few fetches; totals agree to 1e-3
    for a, b in [(st.rays, cnt.rays), (st.node_fetch, cnt.nodes), (st.tri_fetch, cnt.tris),
                 (st.mat_fetch, cnt.mats), (st.tex_fetch, cnt.texels)]:
        assert abs(a - b) <= 1e-3 * b + 2, (a, b)


@pytest.mark.parametrize("name,integrator", [("c2", "lambert"), ("c3", "disney"), ("c3", "mis"), ("c4", "mis")])
def test_frame_kernels_agree(request, name, integrator):
    """The lock-step megakernel (FLAG_MEGAKERNEL; the default for Disney/MIS on small scenes),
    the path-regeneration kernel (FLAG_REGEN) and its large-scene form (the default for Lambert:
    4-wide walk with dynamic ray fetch, camera-ray pass) give bit-identical images. (The staged
    wavefront pipeline, FLAG_WAVEFRONT, was retired in round 5: pt_create rejects it.)"""
    from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_REGEN, FLAG_WAVEFRONT
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    mb = {"disney": 5}.get(integrator, cfg.max_bounce)
    a, sa = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator=integrator, max_bounce=mb, flags=FLAG_REGEN)
    b, sb = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator=integrator, max_bounce=mb, flags=FLAG_MEGAKERNEL)
    d, sd = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator=integrator, max_bounce=mb)
    e, se = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator=integrator, max_bounce=mb, stream=True)
    # streams of frames run the regen kernel by default for Lambert and MIS at its shader's own 2
    # bounces (pt_runtime.cpp regenAll); a synchronous display() call's single frame the megakernel
    assert sb.regen == 0 and sd.regen == 0
    assert se.regen == (1 if integrator == "lambert" or (integrator == "mis" and mb <= 2) else 0)
    if integrator == "mis" and se.regen:  # the MIS wide kernel on a scene that fits the L2s: 3 waves/SIMD
        assert se.waves_per_simd == 3
    assert np.array_equal(a, b)
    assert np.array_equal(d, b)
    assert np.array_equal(e, b)
    if integrator == "mis":
        # regeneration skips BRDF rays whose pdf is 0 (IS:816 discards them after tracing)
        assert sb.rays >= sa.rays >= 0.95 * sb.rays
    else:
        assert sa.rays == sb.rays == sd.rays
    with pytest.raises(RuntimeError, match="retired"):
        Renderer(64, 64, integrator, flags=FLAG_WAVEFRONT)


@pytest.mark.parametrize("name,integrator", [("c2", "lambert"), ("c3", "disney"), ("c3", "mis"), ("c4", "mis")])
def test_runtime_tree_equals_reference_tree(request, name, integrator):
    """Traversing the runtime's own tree (a binned-SAH build; results checked against the
    uploaded tree and retraced through it on a tie or an unreachable hit) gives the image of
    the uploaded reference tree bit for bit, with the same rays, over several frames."""
    from opengl_ray_tracing_amd import FLAG_REFERENCE_TREE
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    mb = {"disney": 5}.get(integrator, cfg.max_bounce)
    a, sa = render_gpu(cfg, tris, nodes, hdr, frames=3, integrator=integrator, max_bounce=mb)
    b, sb = render_gpu(cfg, tris, nodes, hdr, frames=3, integrator=integrator, max_bounce=mb,
                       flags=FLAG_REFERENCE_TREE)
    assert np.array_equal(a, b)
    assert sa.rays == sb.rays


def test_tile_splitting_does_not_change_the_image(c4):
    """Long-path tiles split into smaller work items (frames 4-10 after a restart, while the
    runtime probes the split policy; frames issued serially -- launches that batch frames never
    split) only regroup lanes: the image equals the fixed-order, one-item-per-tile one bit for bit,
    with the same rays, and splitting did happen."""
    from opengl_ray_tracing_amd import FLAG_NO_TILE_ORDER, FLAG_SERIAL_FRAMES
    cfg, tris, nodes, hdr = c4
    eye, rot = orbit_camera(*cfg.camera)
    split_seen = 0
    with Renderer(W, H, cfg.integrator, max_bounce=cfg.max_bounce, flags=FLAG_SERIAL_FRAMES) as r:
        r.upload_scene(tris, nodes)
        r.upload_env(hdr)
        for f in range(12):
            r.render_frame(eye, rot, f)
            split_seen = max(split_seen, r.stats().split_items)
        a, sa = r.accum(), r.stats()
    b, sb = render_gpu(cfg, tris, nodes, hdr, frames=12, flags=FLAG_NO_TILE_ORDER)
    assert split_seen > 0
    assert np.array_equal(a, b)
    assert sa.rays == sb.rays


def test_tile_order_does_not_change_the_image(c4):
    """Longest-tiles-first scheduling (default) only reorders work: frames after the first use the
    previous frame's per-tile costs, and the image equals the fixed-order one bit for bit."""
    from opengl_ray_tracing_amd import FLAG_NO_TILE_ORDER
    cfg, tris, nodes, hdr = c4
    a, sa = render_gpu(cfg, tris, nodes, hdr, frames=3)
    b, sb = render_gpu(cfg, tris, nodes, hdr, frames=3, flags=FLAG_NO_TILE_ORDER)
    assert np.array_equal(a, b)
    assert sa.rays == sb.rays


def test_large_scene_runs_the_wide_kernel_and_matches_oracle():
    """A scene past PT_WIDE_SCENE_MB (216k triangles here, like c5's heightfield + teapot)
    runs the MIS path-regeneration kernel compiled for 4 waves/SIMD by default, and the MIS
    megakernel compiled for 3 with FLAG_MEGAKERNEL; its pixels meet the oracle's under the
    same tolerance as test_render_parity, and every kernel and tree gives the same image."""
    from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_REFERENCE_TREE
    s = scenes.scene_c3()
    v, i = scenes.heightfield(330)
    s.add_mesh(v, i, scenes.Material(baseColor=(0.6, 0.6, 0.65), roughness=0.4, metallic=0.2, specular=0.5),
               scenes.get_transform_matrix((0, 0, 0), (0, -1.2, 0), (13.0, 13.0, 13.0)), True)
    s.build_bvh("binned", 8)
    tris, nodes = s.encode()
    assert tris.size // 36 > 210000
    cfg = scenes.CONFIGS["c5"]
    hdr = scenes.load_hdr(scenes.HDR_FILES[cfg.env])
    w, h, mb = 160, 90, 4
    g, st = render_gpu(cfg, tris, nodes, hdr, frames=2, max_bounce=mb, w=w, h=h)
    assert st.regen == 1 and st.waves_per_simd == 4
    m, sm = render_gpu(cfg, tris, nodes, hdr, frames=2, max_bounce=mb, w=w, h=h, flags=FLAG_MEGAKERNEL)
    assert sm.regen == 0 and sm.waves_per_simd == 3
    b, sb = render_gpu(cfg, tris, nodes, hdr, frames=2, max_bounce=mb, w=w, h=h,
                       flags=FLAG_MEGAKERNEL | FLAG_REFERENCE_TREE)
    assert np.array_equal(g, m) and np.array_equal(m, b) and sm.rays == sb.rays
    # regeneration skips BRDF rays whose pdf is 0 (IS:816 discards them after tracing)
    assert sm.rays >= st.rays >= 0.95 * sm.rays
    px = parity.sample_pixels(w, h, w * h, seed=3)
    o, _ = render_oracle(cfg, tris, nodes, hdr, px, frames=2, max_bounce=mb, w=w, h=h)
    parity.assert_parity(g[px[:, 1], px[:, 0]], o[px[:, 1], px[:, 0]], "wide/mis")
    assert np.all(g[..., 3] == 1.0)
    # the uniform Disney integrator (D:443-481) takes the same large-scene kernel, and so does
    # Lambert (on every scene)
    d, sd = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator="disney", max_bounce=mb, w=w, h=h)
    dm, sdm = render_gpu(cfg, tris, nodes, hdr, frames=2, integrator="disney", max_bounce=mb, w=w, h=h,
                         flags=FLAG_MEGAKERNEL)
    assert sd.regen == 1 and sdm.regen == 0
    assert np.array_equal(d, dm) and sd.rays == sdm.rays
    od, _ = render_oracle(cfg, tris, nodes, hdr, px, frames=2, integrator="disney", max_bounce=mb, w=w, h=h)
    parity.assert_parity(d[px[:, 1], px[:, 0]], od[px[:, 1], px[:, 0]], "wide/disney")
    _, sl = render_gpu(cfg, tris, nodes, hdr, frames=1, integrator="lambert", max_bounce=mb, w=w, h=h)
    assert sl.regen == 1


@pytest.mark.parametrize("name,tile,depth", [("c4", (0, 1), None), ("c2", (1, 3), None), ("c4", (0, 1), 3),
                                              ("c2", (1, 3), 8), ("c2m", (0, 1), None)])
def test_pipelined_frames_equal_serial_frames(request, monkeypatch, name, tile, depth):
    """Frames in flight (the default: frame f+1's megakernel overlaps frame f's tail, each
    frame's running-mean update runs in frame order) give the image of serial frames
    (PT_FLAG_SERIAL_FRAMES) bit for bit -- through the policy probes (the depth probe drains
    and changes the pipeline depth mid-stream), a camera reset, images read mid-stream and a
    screen-tile shard, and at fixed depths 3 and 8 (PT_PIPE_DEPTH) -- with the same rays."""
    from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_SERIAL_FRAMES
    if depth is not None:
        monkeypatch.setenv("PT_PIPE_DEPTH", str(depth))
    extra = 0
    if name == "c2m":  # c2 through the megakernel (Lambert defaults to the regen kernel)
        name, extra = "c2", FLAG_MEGAKERNEL
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    eye, rot = orbit_camera(*cfg.camera)
    eye2, rot2 = orbit_camera(30.0, 15.0, 4.0)
    w, h = 960, 540
    frames = [(eye, rot, f) for f in range(24)] + [(eye2, rot2, f) for f in range(20)]

    def run(flags):
        out = []
        with Renderer(w, h, cfg.integrator, max_bounce=cfg.max_bounce, flags=flags | extra, tile_rank=tile[0],
                      tile_world=tile[1]) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for k, (e, m, f) in enumerate(frames):
                r.render_frame(e, m, f, sync=False)
                if k in (10, 20, 30):
                    out.append(r.accum())
            out.append(r.accum())
            return out, r.stats()

    a, sa = run(0)
    b, sb = run(FLAG_SERIAL_FRAMES)
    assert sa.frames_in_flight == (depth or sa.frames_in_flight) and sa.frames_in_flight >= 2
    assert sb.frames_in_flight == 1
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert sa.rays == sb.rays


@pytest.mark.parametrize("name,tile,batch,flags", [("c4", (0, 8), 0, 0), ("c2", (3, 8), 0, 0), ("c2", (0, 1), 3, 0),
                                                   ("c4", (1, 4), 4, "primary"), ("c2m", (0, 8), 8, 0),
                                                   ("c3", (2, 8), 5, "regen")])
def test_frame_batches_equal_serial_frames(request, name, tile, batch, flags):
    """Batches of frames (pt_render_frames_async: several frames of one camera per launch, their
    running-mean updates applied together pixel by pixel in frame order) give the images and ray
    counts of serial frames bit for bit: small screen-tile shares (the automatic batch, tile_world
    frames), a whole frame, the camera-ray pass, the megakernel and the regen kernel, batches that
    straddle the policy probe and a camera restart, images read between batches and after a clear."""
    from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_PRIMARY_PASS, FLAG_REGEN, FLAG_SERIAL_FRAMES
    extra = {"primary": FLAG_PRIMARY_PASS | FLAG_MEGAKERNEL, "regen": FLAG_REGEN}.get(flags, 0)
    if name == "c2m":
        name, extra = "c2", FLAG_MEGAKERNEL
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    eye, rot = orbit_camera(*cfg.camera)
    eye2, rot2 = orbit_camera(30.0, 15.0, 4.0)
    w, h = 960, 540
    # (camera, first frame, frames): the probe's frames, then batches of varied sizes, a restart
    calls = [((eye, rot), 0, 7), ((eye, rot), 7, 16), ((eye, rot), 23, 9), ((eye, rot), 32, 24),
             ((eye2, rot2), 0, 1), ((eye2, rot2), 1, 30), ((eye2, rot2), 31, 11)]

    def run(fl, batched):
        out = []
        with Renderer(w, h, cfg.integrator, max_bounce=cfg.max_bounce, flags=fl | extra, tile_rank=tile[0],
                      tile_world=tile[1], frame_batch=batch) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for k, ((e, m), f0, n) in enumerate(calls):
                if batched:
                    r.render_frames(e, m, f0, n)
                else:
                    for f in range(f0, f0 + n):
                        r.render_frame(e, m, f, sync=False)
                if k in (2, 3, 5):
                    out.append(r.accum())
                if k == 3:
                    r.clear()
            out.append(r.accum())
            return out, r.stats()

    a, sa = run(0, True)
    b, sb = run(FLAG_SERIAL_FRAMES, False)
    assert sa.frames == sb.frames == sum(c[2] for c in calls)
    few = sa.frames_in_flight <= 3  # pt_runtime.cpp batchFor: few hardware queues, more frames per launch
    mis = 32 if cfg.max_bounce > 2 else 16  # MIS beyond 2 bounces: the megakernel's batches
    m = (12 if few else 2) if cfg.integrator == "lambert" else (mis if few else 4)
    auto = min(m * tile[1], 32)
    assert sa.frame_batch == (batch or auto) and sa.launches < sa.frames
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert sa.rays == sb.rays


@pytest.mark.parametrize("name,integrator,tile", [("c2", "lambert", (0, 1)), ("c3", "mis", (0, 1)),
                                                  ("c4", "mis", (0, 1)), ("c2", "lambert", (2, 3))])
def test_camera_bins_equal_bvh_camera_rays(request, name, integrator, tile):
    """Camera rays found through the per-tile camera-ray bins (the default; pt_primary.hip)
    give the images of camera rays that walk the BVH (PT_FLAG_NO_BINS) bit for bit, with
    the same rays -- across a camera move (the bins are rebuilt) and on a screen-tile shard."""
    from opengl_ray_tracing_amd import FLAG_NO_BINS
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    cams = [orbit_camera(*cfg.camera), orbit_camera(40.0, 25.0, 3.0), orbit_camera(-70.0, -10.0, 6.0)]
    w, h = 960, 540

    def run(flags):
        out = []
        with Renderer(w, h, integrator, max_bounce=cfg.max_bounce, flags=flags, tile_rank=tile[0],
                      tile_world=tile[1]) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for e, m in cams:
                for f in range(3):
                    r.render_frame(e, m, f, sync=False)
                out.append(r.accum())
            return out, r.stats()

    a, sa = run(0)
    b, sb = run(FLAG_NO_BINS)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert sa.rays == sb.rays


@pytest.mark.parametrize("name,integrator,tile,regen", [("c2", "lambert", (0, 1), False), ("c4", "mis", (0, 1), False),
                                                        ("c3", "disney", (1, 3), False), ("c4", "mis", (0, 1), True),
                                                        ("c3", "disney", (1, 3), True)])
def test_camera_ray_pass_equals_megakernel_camera_rays(request, name, integrator, tile, regen):
    """The camera-ray pass (primaryKernel, one wave per tile before the frame kernel,
    PT_FLAG_PRIMARY_PASS) gives the images and ray counts of camera rays traced inside the
    megakernel / the path-regeneration kernel bit for bit: near and far cameras (the far one
    fills bins past PT_BIN_CAP, whose tiles the frame kernel traces itself), a camera move and
    a shard."""
    from opengl_ray_tracing_amd import FLAG_MEGAKERNEL, FLAG_PRIMARY_PASS, FLAG_REGEN
    cfg, tris, nodes, hdr = request.getfixturevalue(name)
    cams = [orbit_camera(*cfg.camera), orbit_camera(40.0, 25.0, 1.5), orbit_camera(-70.0, -10.0, 14.0)]
    w, h = 960, 540

    def run(flags):
        out = []
        with Renderer(w, h, integrator, max_bounce=cfg.max_bounce, flags=flags, tile_rank=tile[0],
                      tile_world=tile[1]) as r:
            r.upload_scene(tris, nodes)
            r.upload_env(hdr)
            for e, m in cams:
                for f in range(3):
                    r.render_frame(e, m, f, sync=False)
                out.append(r.accum())
            return out, r.stats()

    base = FLAG_REGEN if regen else FLAG_MEGAKERNEL
    a, sa = run(base)
    b, sb = run(base | FLAG_PRIMARY_PASS)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert sa.rays == sb.rays
