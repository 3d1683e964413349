"""Host scene preparation: readObj semantics (OpenglRayTracing/main.cpp:261-372),
getTransformMatrix (:242-258), the display() camera (:569-573), the BVH
builders (:376-551) and the encoded layout (:687-716)."""
import numpy as np
import pytest

from opengl_ray_tracing_amd import Material, Scene, get_transform_matrix, orbit_camera, scenes

BUILDERS = ["sah", "median", "fixed_sah", "binned"]


def f32(x):
    return np.float32(x)


def test_transform_matrix_matches_glm_composition():
    M = get_transform_matrix((0, 0, 0), (0.3, -1.6, 0), (1.5, 1.5, 1.5)).reshape(4, 4).T  # row-major view
    want = np.array([[1.5, 0, 0, 0.3], [0, 1.5, 0, -1.6], [0, 0, 1.5, 0], [0, 0, 0, 1]], np.float32)
    assert np.array_equal(M, want)
    R = get_transform_matrix((0, 90, 0), (0, 0, 0), (1, 1, 1)).reshape(4, 4).T
    assert np.allclose(R[:3, :3], [[0, 0, 1], [0, 1, 0], [-1, 0, 0]], atol=1e-6)


def test_orbit_camera_is_inverse_lookat():
    for rot, up, r in [(0, 0, 4), (30, 20, 5.5), (-120, -60, 3)]:
        eye, cam = orbit_camera(rot, up, r)
        th, ph = np.radians(up), np.radians(rot)
        want_eye = r * np.array([-np.sin(ph) * np.cos(th), np.sin(th), np.cos(ph) * np.cos(th)])
        assert np.allclose(eye, want_eye, atol=1e-5)
        C = cam.reshape(4, 4).T
        f = -eye / np.linalg.norm(eye)
        s = np.cross(f, [0, 1, 0])
        s /= np.linalg.norm(s)
        u = np.cross(s, f)
        assert np.allclose(C[:3, 0], s, atol=1e-5) and np.allclose(C[:3, 1], u, atol=1e-5)
        assert np.allclose(C[:3, 2], -f, atol=1e-5) and np.allclose(C[:3, 3], eye, atol=1e-4)


def test_read_obj_aabb_typo_and_normals():
    # readObj normalises by max(lenx, leny, lenz) where maxy/maxz/miny/minz track the running x
    # extremes (main.cpp:297-298); the last vertex decides leny/lenz.
    text = "v 0 0 0\nv 4 0 0\nv 0 1 0\nv 0 0 1\nf 1 2 3\nf 1/1 2/2 4/4\nf 1/1/1 3/3/3 4/4/4\n"
    s = Scene()
    s.read_obj_text(text, Material(), None, False)
    tris, _ = s.encode()
    assert tris.shape == (3, 36)
    # maxx=4, minx=0 -> maxy=max(4,0)=4, miny=min(0,0)=0, ... maxaxis = 4
    assert np.array_equal(tris[0, 0:9], np.array([0, 0, 0, 1, 0, 0, 0, 0.25, 0], np.float32))
    # flat normals: normalize(cross(p2-p1, p3-p1))
    assert np.allclose(tris[0, 9:12], [0, 0, 1])
    assert np.array_equal(tris[0, 9:18], np.tile(tris[0, 9:12], 3))
    # smooth: vertex normals = normalized sum of adjacent face normals
    s2 = Scene()
    s2.read_obj_text(text, Material(), None, True)
    t2, _ = s2.encode()
    n = t2[0, 9:12]
    assert np.allclose(np.linalg.norm(n), 1, atol=1e-6)
    # material encode (main.cpp:701-706)
    m = Material(emissive=(1, 2, 3), baseColor=(0.1, 0.2, 0.3), subsurface=0.1, metallic=0.2, specular=0.3,
                 specularTint=0.4, roughness=0.5, anisotropic=0.6, sheen=0.7, sheenTint=0.8, clearcoat=0.9,
                 clearcoatGloss=0.95, IOR=1.5, transmission=0.25)
    s3 = Scene()
    s3.read_obj_text(text, m, None, False)
    t3, _ = s3.encode()
    assert np.array_equal(t3[0, 18:36], np.array([1, 2, 3, 0.1, 0.2, 0.3, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8,
                                                  0.9, 0.95, 1.5, 0.25], np.float32))


def test_add_mesh_equals_read_obj():
    v, i = scenes.uv_sphere(8, 6, lambda u, w: 1.0)
    text = "".join(f"v {float(x)!r} {float(y)!r} {float(z)!r}\n" for x, y, z in v) + \
        "".join(f"f {a + 1} {b + 1} {c + 1}\n" for a, b, c in i)
    T = get_transform_matrix((10, 20, 30), (0.5, -1, 2), (2, 3, 4))
    a, b = Scene(), Scene()
    a.add_mesh(v, i, Material(), T, True)
    b.read_obj_text(text, Material(), T, True)
    ta, _ = a.encode()
    tb, _ = b.encode()
    assert np.array_equal(ta, tb)


def test_read_obj_missing_file_is_an_error():
    with pytest.raises(RuntimeError):
        Scene().read_obj("/nonexistent/bunny.obj", Material())


def check_tree(tris, nodes, leaf):
    n = tris.shape[0]
    # dummy node 0 (main.cpp:675-681)
    assert np.array_equal(nodes[0, [0, 1, 3]], [255, 128, 30])
    assert np.array_equal(nodes[0, 6:12], [1, 1, 0, 0, 1, 0])
    covered = np.zeros(n, np.int32)
    stack, seen, maxd = [(1, 1)], 0, 0
    while stack:
        k, d = stack.pop()
        seen += 1
        maxd = max(maxd, d)
        AA, BB = nodes[k, 6:9], nodes[k, 9:12]
        cnt, idx = int(nodes[k, 3]), int(nodes[k, 4])
        if cnt > 0:
            assert 1 <= cnt <= leaf
            covered[idx:idx + cnt] += 1
            p = tris[idx:idx + cnt, 0:9].reshape(-1, 3)
            assert np.all(p >= AA) and np.all(p <= BB)
        else:
            L, R = int(nodes[k, 0]), int(nodes[k, 1])
            assert 0 < L < len(nodes) and 0 < R < len(nodes)
            for c in (L, R):
                assert np.all(nodes[c, 6:9] >= AA) and np.all(nodes[c, 9:12] <= BB)
                stack.append((c, d + 1))
    assert np.all(covered == 1), "every triangle in exactly one leaf"
    assert seen == len(nodes) - 1
    return maxd


@pytest.mark.parametrize("builder", BUILDERS)
def test_bvh_builders_produce_valid_trees(builder):
    s = scenes.scene_c2()
    s.build_bvh(builder, 8)
    tris, nodes = s.encode()
    d = check_tree(tris, nodes, 8)
    assert d == s.depth
    # node ids in preorder: children have larger ids
    internal = nodes[1:][nodes[1:, 3] <= 0]
    assert np.all(internal[:, 0] > 0)


def test_reference_sah_typo_changes_only_the_tree():
    a, b = scenes.scene_c2(), scenes.scene_c2()
    a.build_bvh("sah", 8)
    b.build_bvh("fixed_sah", 8)
    ta, na = a.encode()
    tb, nb = b.encode()
    key = lambda t: np.lexsort(t[:, :9].T)  # noqa: E731
    assert np.array_equal(ta[key(ta)], tb[key(tb)])
    assert a.depth > b.depth  # typo'd trees are much deeper (depth 55 vs 10-13 at 5k tris)


def test_builders_are_deterministic():
    out = []
    for _ in range(2):
        s = scenes.scene_c4()
        s.build_bvh("sah", 8)
        out.append(s.encode())
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


def test_scene_sizes():
    s = scenes.scene_c2()
    assert s.num_triangles == 5004  # 5,000-triangle bunny stand-in + 2 quads
    t = scenes.scene_c3()
    assert 6000 <= t.num_triangles <= 6700


def test_heightfield_triangle_count():
    v, i = scenes.heightfield(708)
    assert i.shape[0] == 999_698
    assert v.shape[0] == 708 * 708


def test_cornell_shapes():
    sh = scenes.cornell_shapes()
    assert sh.shape == (17, 24)
    assert np.sum(sh[:, 0] == 1) == 3  # spheres
    assert np.sum(sh[:, 16] == 1) == 2  # emissive light triangles
    tri = sh[sh[:, 0] == 0]
    assert np.allclose(np.linalg.norm(tri[:, 13:16], axis=1), 1, atol=1e-6)


# sha1 of encode() for a 39,762-triangle heightfield, produced by the serial
# (single-threaded) builders before the threaded build existed: subtrees above
# 8,192 triangles are now built on their own threads and spliced back in
# preorder, which must not change a single bit of the arrays.
SERIAL_BUILD_SHA1 = {
    "median": "90c51138bb41f6d860d12280873309b00ed61797",
    "fixed_sah": "9fd2b6ece29ee6806aa6321cffbf93c8092a5ee4",
    "binned": "61b7d43dc35f341155d574a9e3562cb1f277715e",
}


@pytest.mark.parametrize("builder", sorted(SERIAL_BUILD_SHA1))
def test_threaded_build_equals_serial_build(builder):
    import hashlib
    from opengl_ray_tracing_amd.scene import Material, Scene
    v, i = scenes.heightfield(142)
    s = Scene()
    s.add_mesh(v, i, Material())
    s.build_bvh(builder, 8)
    t, n = s.encode()
    check_tree(t, n, 8)
    assert hashlib.sha1(t.tobytes() + n.tobytes()).hexdigest() == SERIAL_BUILD_SHA1[builder]
