"""Parity metrics shared by the GPU tests (test infrastructure).

Tolerances (DESIGN.md "Parity"): float32 path tracing where +,-,*,/,sqrt round
identically on both sides and the transcendentals (ocml vs glibc) may differ
by ~1 ulp. A 1-ulp difference can flip a discrete branch (edge hit, lobe
choice, Russian roulette) and change a 1-spp pixel completely, so the bar is:
  * per-pixel relative L2 <= 1e-3 on >= 99.9 % of compared pixels,
  * image-mean relative L2 <= 1e-4 over the compared pixels.
"""
from __future__ import annotations

import numpy as np

PIX_TOL = 1e-3
PIX_FRAC = 0.999
MEAN_TOL = 1e-4


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


def assert_parity(g, o, what=""):
    s = summary(g, o)
    assert s["finite"], f"{what}: non-finite GPU values {s}"
    assert s["within"] >= PIX_FRAC, f"{what}: per-pixel parity {s}"
    assert s["mean_rel"] <= MEAN_TOL, f"{what}: image-mean parity {s}"
    return s


def sample_pixels(w: int, h: int, n: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    k = rng.choice(w * h, size=min(n, w * h), replace=False)
    return np.stack([k % w, k // w], 1).astype(np.int32)
