"""Image output (include/pt_scene.h): PFM of the linear accumulation and the
8-bit PNG of BasicRayTracingWithC++'s imshow (main.cpp:169-190)."""
import numpy as np

from opengl_ray_tracing_amd import read_pfm, write_pfm, write_png


def _img(h=37, w=53, c=4, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.gamma(0.7, 0.6, size=(h, w, c)).astype(np.float32)
    a[0, 0, 0] = -1.0  # clamped
    a[1, 1, 1] = 50.0
    return a


def test_pfm_roundtrip(tmp_path):
    a = _img()
    write_pfm(tmp_path / "a.pfm", a)
    b = read_pfm(tmp_path / "a.pfm")
    assert np.array_equal(b, a[..., :3])


def test_png_is_imshow(tmp_path):
    from PIL import Image
    a = _img(c=3)
    write_png(tmp_path / "a.png", a, gamma=2.2, flip_rows=True)
    got = np.asarray(Image.open(tmp_path / "a.png"))
    with np.errstate(invalid="ignore"):
        v = np.power(a.astype(np.float64), np.float64(np.float32(1) / np.float32(2.2))) * 255
    want = np.clip(np.nan_to_num(v, nan=0.0), 0, 255).astype(np.uint8)[::-1]
    assert got.shape == (37, 53, 3)
    assert np.array_equal(got, want)


def test_png_large_spans_stored_blocks(tmp_path):
    from PIL import Image
    a = np.linspace(0, 1, 300 * 400 * 3, dtype=np.float32).reshape(300, 400, 3)
    write_png(tmp_path / "b.png", a, gamma=0.0, flip_rows=False)
    got = np.asarray(Image.open(tmp_path / "b.png"))
    assert np.array_equal(got, np.clip(a.astype(np.float64) * 255, 0, 255).astype(np.uint8))
