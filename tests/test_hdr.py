"""HDR environment: Radiance decode (hdrloader.cpp:29-191) and the importance
sampling cache (calculateHdrCache, IS main.cpp:555-652).

Pinned by (i) an independent decoder of the Radiance RLE format written here,
(ii) the statistics SURVEY.md 8(c) recorded from the reference's own
HDRLoader compiled in this container (peppermint 1024x512 mean (0.3077,
0.2924, 0.3106) max 21; san_giuseppe 2048x1024 mean (0.7135, 0.6494, 0.5747)
max 354), and (iii) the CPU restatement of calculateHdrCache in oracle/."""
import numpy as np
import pytest

import oracle
from opengl_ray_tracing_amd import calculate_hdr_cache, decode_hdr, load_hdr, scenes


def decode_independent(data: bytes) -> np.ndarray:
    i = data.index(b"\n\n") + 2
    j = data.index(b"\n", i)
    _, h, _, w = data[i:j].decode().split()
    h, w = int(h), int(w)
    i = j + 1
    out = np.zeros((h, w, 4), np.uint8)
    for y in range(h):
        assert data[i] == 2 and data[i + 1] == 2
        i += 4
        for c in range(4):
            x = 0
            while x < w:
                code = data[i]
                i += 1
                if code > 128:
                    out[y, x:x + code - 128, c] = data[i]
                    i += 1
                    x += code - 128
                else:
                    out[y, x:x + code, c] = np.frombuffer(data[i:i + code], np.uint8)
                    i += code
                    x += code
    e = out[..., 3].astype(np.int32) - 128
    return (out[..., :3].astype(np.float32) / np.float32(256.0)) * np.ldexp(np.float32(1), e)[..., None].astype(
        np.float32)


@pytest.mark.parametrize("name,shape,mean,mx", [
    ("peppermint", (512, 1024, 3), (0.3077, 0.2924, 0.3106), 21.0),
    ("san_giuseppe", (1024, 2048, 3), (0.7135, 0.6494, 0.5747), 354.0),
])
def test_decode_matches_reference_loader_stats(name, shape, mean, mx):
    img = load_hdr(scenes.HDR_FILES[name])
    assert img.shape == shape
    m = img.reshape(-1, 3).astype(np.float64).mean(0)
    assert np.allclose(m, mean, atol=6e-5)
    assert img.max() == mx


@pytest.mark.parametrize("name", ["peppermint", "san_giuseppe"])
def test_decode_bit_exact_vs_independent_decoder(name):
    data = scenes.HDR_FILES[name].read_bytes()
    assert np.array_equal(decode_hdr(data), decode_independent(data))


def test_decode_rejects_garbage():
    with pytest.raises(RuntimeError):
        decode_hdr(b"not a radiance file at all")
    with pytest.raises(RuntimeError):
        load_hdr("/nonexistent.hdr")


def test_old_rle_and_flat_scanlines():
    # width < 8 uses the old (uncompressed/old-RLE) scanline path (hdrloader.cpp:122-123)
    w, h = 4, 2
    px = bytes([128, 64, 32, 129, 1, 1, 1, 2, 255, 0, 0, 128])
    data = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 2 +X 4\n" + px + px
    img = decode_hdr(data)
    assert img.shape == (h, w, 3)
    assert np.allclose(img[0, 0], np.array([128, 64, 32]) / 256.0 * 2.0)
    # (1,1,1,e) repeats the previous pixel e << rshift times
    assert np.array_equal(img[0, 1], img[0, 0]) and np.array_equal(img[0, 2], img[0, 0])
    assert np.allclose(img[0, 3], np.array([255, 0, 0]) / 256.0)


def test_hdr_cache_matches_oracle_restatement():
    for hdr in [scenes.synthetic_env(64, 32), load_hdr(scenes.HDR_FILES["peppermint"])]:
        a = calculate_hdr_cache(hdr)
        b = oracle.hdr_cache(hdr)
        assert np.array_equal(a, b)


def test_hdr_cache_properties():
    hdr = load_hdr(scenes.HDR_FILES["peppermint"])
    c = calculate_hdr_cache(hdr)
    assert np.all((c[..., 0] >= 0) & (c[..., 0] <= 1)) and np.all((c[..., 1] >= 0) & (c[..., 1] <= 1))
    # pdf = lum / lumSum with lumSum accumulated in float32 in scanline order (IS main.cpp:557-576)
    hd = hdr.astype(np.float64)
    lum = (0.2 * hd[..., 0] + 0.7 * hd[..., 1] + 0.1 * hd[..., 2]).astype(np.float32)
    lum_sum = np.cumsum(lum.ravel(), dtype=np.float32)[-1]
    assert np.array_equal(c[..., 2], lum / lum_sum)
    assert abs(float(c[..., 2].astype(np.float64).sum()) - 1.0) < 1e-3
    # sampled columns follow the marginal: bright columns are sampled more often
    xs = np.round(c[..., 0] * hdr.shape[1]).astype(int).ravel()
    hist = np.bincount(np.clip(xs, 0, hdr.shape[1] - 1), minlength=hdr.shape[1]).astype(np.float64)
    marg = lum.sum(0) / lum.sum()
    assert np.corrcoef(hist / hist.sum(), marg)[0, 1] > 0.9
