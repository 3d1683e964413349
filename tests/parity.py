"""Parity metrics shared by the GPU tests (test infrastructure).

What is asserted: the GPU and the CPU restatement evaluate the same
float32 operations in the same order (+,-,*,/,sqrt IEEE on both sides, the
transcendentals from the one shared include/pt_fmath.h), so images are equal BIT FOR
BIT -- `exact == 1.0` is asserted by default, which is what README/DESIGN claim.
The stated tolerance bar of SURVEY.md 8(c) / BASELINE.md is asserted as well and
reported in every failure message, so a regression shows how far it is off:
  * per-pixel relative L2 <= 1e-3 on >= 99.9 % of compared pixels,
  * image-mean relative L2 <= 1e-4 over the compared pixels,
  * linear PSNR >= 60 dB (peak = the oracle image's maximum; inf when exact).
A case that is not bit-exact by construction passes exact=False and keeps the bar.
"""
from __future__ import annotations

import numpy as np

PIX_TOL = 1e-3
PIX_FRAC = 0.999
MEAN_TOL = 1e-4
PSNR_MIN_DB = 60.0


def rel_l2(g: np.ndarray, o: np.ndarray) -> np.ndarray:
    g = np.asarray(g, np.float64)[..., :3]
    o = np.asarray(o, np.float64)[..., :3]
    num = np.linalg.norm(g - o, axis=-1)
    den = np.maximum(np.linalg.norm(o, axis=-1), 1e-6)
    return num / den


def summary(g: np.ndarray, o: np.ndarray) -> dict:
    r = rel_l2(g, o)
    g3 = np.asarray(g, np.float64)[..., :3]
    o3 = np.asarray(o, np.float64)[..., :3]
    mean_rel = abs(g3.mean() - o3.mean()) / max(abs(o3.mean()), 1e-12)
    mse = np.mean((g3 - o3) ** 2)
    peak = max(o3.max(), 1e-12)
    psnr = float("inf") if mse == 0 else 10 * np.log10(peak ** 2 / mse)
    return {
        "n": int(r.size),
        "exact": float(np.mean(np.all(g3 == o3, axis=-1))),
        "within": float(np.mean(r <= PIX_TOL)),
        "max_rel": float(r.max()) if r.size else 0.0,
        "mean_rel": float(mean_rel),
        "psnr": float(psnr),
        "finite": bool(np.isfinite(np.asarray(g)).all()),
    }


def assert_parity(g, o, what="", exact=True):
    s = summary(g, o)
    bar = f"(bar: within {PIX_TOL} on >= {PIX_FRAC}, mean <= {MEAN_TOL}, PSNR >= {PSNR_MIN_DB} dB)"
    assert s["finite"], f"{what}: non-finite GPU values {s}"
    assert s["within"] >= PIX_FRAC, f"{what}: per-pixel parity {s} {bar}"
    assert s["mean_rel"] <= MEAN_TOL, f"{what}: image-mean parity {s} {bar}"
    assert s["psnr"] >= PSNR_MIN_DB, f"{what}: linear PSNR {s} {bar}"
    if exact:
        assert s["exact"] == 1.0, f"{what}: not bit-exact against the oracle {s} {bar}"
    return s


def sample_pixels(w: int, h: int, n: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    k = rng.choice(w * h, size=min(n, w * h), replace=False)
    return np.stack([k % w, k // w], 1).astype(np.int32)
