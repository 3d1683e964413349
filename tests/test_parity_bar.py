"""The parity helper itself (CPU): it asserts bit-exactness by default, the stated
tolerance bar (per-pixel relative L2 <= 1e-3 on >= 99.9 % of pixels,
image mean <= 1e-4) and BASELINE.md's linear PSNR >= 60 dB."""
import numpy as np
import pytest

import parity


def _img(seed=0, n=4096):
    return np.random.default_rng(seed).uniform(0.1, 2.0, (n, 4)).astype(np.float32)


def test_exact_images_pass_with_infinite_psnr():
    a = _img()
    s = parity.assert_parity(a, a.copy(), "same")
    assert s["exact"] == 1.0 and s["psnr"] == float("inf")


def test_one_ulp_off_fails_the_exact_bar_but_not_the_tolerance():
    a = _img()
    b = a.copy()
    b[17, 0] = np.nextafter(b[17, 0], np.float32(10))
    with pytest.raises(AssertionError, match="not bit-exact"):
        parity.assert_parity(b, a, "ulp")
    s = parity.assert_parity(b, a, "ulp", exact=False)
    assert s["within"] == 1.0 and s["psnr"] > parity.PSNR_MIN_DB


def test_psnr_bar_is_enforced():
    a = _img()
    b = a.copy()
    b[0, :3] += 0.2  # two pixels off in opposite directions: within-fraction and mean pass, PSNR does not
    b[1, :3] -= 0.2
    s = parity.summary(b, a)
    assert s["within"] >= parity.PIX_FRAC and s["mean_rel"] <= parity.MEAN_TOL and s["psnr"] < parity.PSNR_MIN_DB
    with pytest.raises(AssertionError, match="linear PSNR"):
        parity.assert_parity(b, a, "psnr", exact=False)
