"""include/pt_fmath.h: the shared transcendentals are the correctly rounded float values
(float64 numpy, i.e. glibc's double functions, rounded to float), special values, and their
distance from glibc's own float functions (sinf ... powf)."""
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


N = 400_000


def _gen(seed):
    rng = np.random.default_rng(seed)
    return rng


# (fn id, name, glibc float function, input generator, float64 reference); the ranges cover every
# use in the kernels (IS:148-149,176,489-490,502-505,525,582,639,660) and beyond
CASES = [
    (0, "sin", "sinf", lambda r, n: (r.uniform(-8, 8, n),), lambda x: np.sin(x[0])),
    (1, "cos", "cosf", lambda r, n: (r.uniform(-8, 8, n),), lambda x: np.cos(x[0])),
    (2, "atan2", "atan2f", lambda r, n: (r.normal(size=n), r.normal(size=n)), lambda x: np.arctan2(x[0], x[1])),
    (3, "asin", "asinf", lambda r, n: (r.uniform(-1, 1, n),), lambda x: np.arcsin(x[0])),
    (4, "log", "logf", lambda r, n: (np.exp(r.uniform(-100, 88, n)),), lambda x: np.log(x[0])),
    (5, "exp", "expf", lambda r, n: (r.uniform(-100, 88, n),), lambda x: np.exp(x[0])),
    (6, "pow", "powf", lambda r, n: (r.uniform(1e-6, 1, n), r.uniform(0, 2, n)), lambda x: np.power(x[0], x[1])),
]


@pytest.mark.parametrize("fn,name,gname,gen,ref", CASES, ids=[c[1] for c in CASES])
def test_correctly_rounded(fn, name, gname, gen, ref):
    """Every value is the float64 result rounded to float (no exception in 4e5 inputs)."""
    x = [a.astype(np.float32) for a in gen(_gen(100 + fn), N)]
    got = host(fn, *x)
    want = ref([a.astype(np.float64) for a in x]).astype(np.float32)
    bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
    assert bad.size == 0, (name, bad.size, [a[bad[:3]] for a in x], got[bad[:3]], want[bad[:3]])


# glibc's float functions are not correctly rounded everywhere: the share of inputs where they
# differ from pt_fmath (always by one ulp), measured on 1e5 inputs of the same ranges
GLIBC_DIFFER_AT_MOST = {"sin": 0.02, "cos": 0.02, "atan2": 0.2, "asin": 0.1, "log": 0.002, "exp": 0.002, "pow": 0.002}


@pytest.mark.parametrize("fn,name,gname,gen,ref", CASES, ids=[c[1] for c in CASES])
def test_distance_from_glibc_float_functions(fn, name, gname, gen, ref):
    m = C.CDLL("libm.so.6")
    x = [a.astype(np.float32) for a in gen(_gen(200 + fn), 100_000)]
    f = getattr(m, gname)
    f.restype = C.c_float
    f.argtypes = [C.c_float] * len(x)
    g = np.array([f(*[float(a[i]) for a in x]) for i in range(x[0].size)], np.float32)
    p = host(fn, *x)
    ulp = np.abs(p.view(np.int32).astype(np.int64) - g.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1, (name, ulp.max())
    assert (ulp > 0).mean() <= GLIBC_DIFFER_AT_MOST[name], (name, (ulp > 0).mean())


def test_special_values():
    a = host(2, np.array([0, 0, 1, -1, 0, -0.0], np.float32), np.array([0, -1, 0, 0, 1, -1], np.float32))
    assert np.allclose(a, [0, np.pi, np.pi / 2, -np.pi / 2, 0, -np.pi], atol=1e-7)
    assert np.isnan(host(3, np.array([1.5], np.float32)))[0]
    assert np.array_equal(host(3, np.array([1, -1], np.float32)), np.float32([np.pi / 2, -np.pi / 2]))
    assert host(4, np.array([1.0], np.float32))[0] == 0.0
    assert host(4, np.array([0.0], np.float32))[0] == -np.inf
    assert host(4, np.array([1e-45], np.float32))[0] == np.float32(np.log(np.float64(np.float32(1e-45))))
    assert host(5, np.array([0.0], np.float32))[0] == 1.0
    assert host(5, np.array([-200.0], np.float32))[0] == 0.0
    assert host(5, np.array([89.0], np.float32))[0] == np.inf
    assert host(6, np.array([0.25], np.float32), np.array([0.5], np.float32))[0] == 0.5
    s = host(0, np.array([0.0, np.pi / 2, np.pi], np.float32))
    assert np.array_equal(s, np.sin(np.float32([0.0, np.pi / 2, np.pi]).astype(np.float64)).astype(np.float32))


def test_ranges_used_by_the_kernel():
    # toSpherical inputs: unit vectors -> |asin arg| <= 1, atan2 on the sphere
    rng = _gen(5)
    v = rng.normal(size=(N, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v = v.astype(np.float32)
    a = host(2, v[:, 2], v[:, 0])
    assert np.all(np.abs(a) <= np.float32(np.pi))
    b = host(3, v[:, 1])
    assert np.all(np.abs(b) <= np.float32(np.pi / 2))
