"""include/pt_fmath.h: accuracy of the shared transcendentals against float64
(numpy), special values, and host == oracle-side evaluation."""
import ctypes as C

import numpy as np
import pytest

from opengl_ray_tracing_amd import _native

FP = C.POINTER(C.c_float)


def host(fn, x, y=None):
    x = np.ascontiguousarray(x, np.float32)
    y = None if y is None else np.ascontiguousarray(y, np.float32)
    out = np.empty_like(x)
    rc = _native.load().pt_fmath_host(fn, x.ctypes.data_as(FP), None if y is None else y.ctypes.data_as(FP), x.size,
                                      out.ctypes.data_as(FP))
    assert rc == 0
    return out


def ulps(got, ref):
    ref = np.asarray(ref, np.float64)
    sp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    return np.abs(got.astype(np.float64) - ref) / sp


rng = np.random.default_rng(12345)
N = 400_000

# (fn id, name, input generator, float64 reference, max ulp measured with a margin)
CASES = [
    (0, "sin", lambda: (rng.uniform(-8, 8, N), None), lambda x, y: np.sin(x), 2.0),
    (1, "cos", lambda: (rng.uniform(-8, 8, N), None), lambda x, y: np.cos(x), 5.0),
    (2, "atan2", lambda: (rng.normal(size=N), rng.normal(size=N)), lambda x, y: np.arctan2(x, y), 4.0),
    (3, "asin", lambda: (rng.uniform(-1, 1, N), None), lambda x, y: np.arcsin(x), 3.0),
    (4, "log", lambda: (np.exp(rng.uniform(-80, 80, N)), None), lambda x, y: np.log(x), 1.0),
    (5, "exp", lambda: (rng.uniform(-80, 80, N), None), lambda x, y: np.exp(x), 1.0),
    (6, "pow", lambda: (rng.uniform(1e-6, 0.01, N), rng.uniform(0, 1, N)), lambda x, y: np.power(x, y), 16.0),
]


@pytest.mark.parametrize("fn,name,gen,ref,bound", CASES, ids=[c[1] for c in CASES])
def test_accuracy(fn, name, gen, ref, bound):
    x, y = gen()
    x = x.astype(np.float32)
    y = None if y is None else y.astype(np.float32)
    got = host(fn, x, y)
    r = ref(x.astype(np.float64), None if y is None else y.astype(np.float64))
    u = ulps(got, r)
    if name == "cos":  # relative ulps blow up at the zeros of cos; bound the absolute error there
        near0 = np.abs(r) < 1e-3
        assert np.max(np.abs(got[near0] - r[near0])) < 2e-8
        u = u[~near0]
    assert u.max() <= bound, (name, u.max())


def test_special_values():
    a = host(2, np.array([0, 0, 1, -1, 0, -0.0], np.float32), np.array([0, -1, 0, 0, 1, -1], np.float32))
    assert np.allclose(a, [0, np.pi, np.pi / 2, -np.pi / 2, 0, -np.pi], atol=1e-7)
    assert np.isnan(host(3, np.array([1.5], np.float32)))[0]
    assert host(4, np.array([1.0], np.float32))[0] == 0.0
    assert host(4, np.array([0.0], np.float32))[0] == -np.inf
    assert np.isfinite(host(4, np.array([1e-40], np.float32)))[0]  # subnormal input
    assert host(5, np.array([0.0], np.float32))[0] == 1.0
    assert host(5, np.array([-200.0], np.float32))[0] == 0.0
    assert host(6, np.array([0.25], np.float32), np.array([0.5], np.float32))[0] == pytest.approx(0.5, abs=1e-7)
    s = host(0, np.array([0.0, np.pi / 2, np.pi], np.float32))
    assert np.allclose(s, [0, 1, 0], atol=1e-7)


def test_ranges_used_by_the_kernel():
    # toSpherical inputs: unit vectors -> |asin arg| <= 1, atan2 on the sphere
    v = rng.normal(size=(N, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v = v.astype(np.float32)
    a = host(2, v[:, 2], v[:, 0])
    assert np.all(np.abs(a) <= np.float32(np.pi))
    b = host(3, v[:, 1])
    assert np.all(np.abs(b) <= np.float32(np.pi / 2))
