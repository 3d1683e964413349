#!/usr/bin/env python3
"""Summarise the megakernel wave lifetimes of a PT_WAVE_TRACE=1 build.

    python tools/tune.py --build wtrace:PT_WAVE_TRACE=1            # here
    PT_WAVE_TRACE_FILE=gpurun_out/w.bin python tools/tune.py --child wtrace --config c4 --frames 3 --warmup 0
    python tools/wave_trace.py gpurun_out/w.bin
    python tools/wave_trace.py --regen gpurun_out/w.bin <waves per frame>   # the regen kernel's records
    python tools/tune.py --build phases:PT_WAVE_TRACE=1,PT_PHASE_STATS=1      # the regen kernel's phases:
    python tools/wave_trace.py --phases gpurun_out/p.bin

Per frame: how long the frame lasted (first wave start to last wave end), how
much of it the average wave was alive, the frame's tail (time from the median
wave end to the last), and the longest single tile.
"""
import sys

import numpy as np


def regen(path, per=None):
    """regenKernel records: start, end, tiles | last lone lane's pixel << 32, last successful claim,
    loop iterations, iterations with at most 4 lanes active."""
    raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 6)
    pix = (raw[:, 2] >> np.uint64(32)).astype(np.int64)
    raw[:, 2] &= np.uint64(0xffffffff)
    a = raw.astype(np.float64)
    n = len(a)
    per = per or n
    us = lambda x: x / 100.0  # 100 MHz ticks -> us
    for f in range(n // per):
        r = a[f * per:(f + 1) * per]
        px = pix[f * per:(f + 1) * per][r[:, 0] > 0]
        r = r[r[:, 0] > 0]
        t0, t1 = r[:, 0].min(), r[:, 1].max()
        drained = r[:, 3].max()  # the last successful claim: every tile handed out
        ends = np.sort(r[:, 1])
        thin = r[:, 5] / np.maximum(r[:, 4], 1)
        print(f"frame {f}: {len(r)} waves, frame {us(t1 - t0):7.1f} us, start spread {us(r[:, 0].max() - t0):6.1f}, "
              f"queues drained at {us(drained - t0):7.1f}, tail after drain {us(t1 - drained):7.1f}, "
              f"median end {us(np.median(ends) - t0):7.1f}, 99% end {us(ends[int(0.99 * len(ends))] - t0):7.1f}, "
              f"tiles/wave {r[:, 2].mean():.1f}, iters/wave {r[:, 4].mean():.0f}, thin iters {thin.mean():.3f}")
        last = np.argsort(-r[:, 1])[:5]
        print("   last waves (end us, iters, thin iters, last lone pixel):",
              ", ".join(f"{us(r[k, 1] - t0):.0f} {r[k, 4]:.0f} {r[k, 5]:.0f} ({px[k] >> 16},{px[k] & 0xffff})"
                        for k in last))


PHASES = ["refill", "walk", "reference check", "shading"]


def phases(path):
    """PT_PHASE_STATS records (pt_regen.hip): 24 u64 per wave, summed over every wave of every frame."""
    raw = np.fromfile(path, dtype=np.uint64).reshape(-1, 24).astype(np.float64)
    raw = raw[raw[:, 15] > 0]
    t = raw.sum(axis=0)
    life = t[15]
    print(f"{len(raw)} wave records, mean lifetime {life / len(raw) / 2.4e3:.1f} us at 2.4 GHz")
    for k, name in enumerate(PHASES):
        print(f"  {name:16s} {t[k] / life:6.3f} of wave time")
    print(f"  (unaccounted      {1 - t[:4].sum() / life:6.3f})")
    it = max(t[4], 1)
    print(f"main-loop iterations with a walk {t[4]:.3g}: lanes walking {t[5] / it:5.1f}, lanes shading {t[6] / it:5.1f}"
          f" (walks cut by the yield {t[12] / it:5.1f} lanes; iterations ending every walk {t[13] / it:.3f})")
    print(f"node iterations {t[7]:.3g} ({t[7] / it:.1f} per walk call), lanes {t[8] / max(t[7], 1):5.1f} of 64")
    print(f"pair tests      {t[9]:.3g} ({t[9] / it:.1f} per walk call), lanes {t[10] / max(t[9], 1):5.1f} of 64")
    print(f"refill iterations {t[11]:.3g}; retraced lanes {t[14]:.3g}")
    if t[17] > 0:  # the uniform integrators' hand-out (TILE_PRIM)
        print(f"  refill = hand-out {t[16] / life:6.3f} (of it tile claims {t[18] / life:6.3f}: {t[17]:.3g} claims, "
              f"{t[18] / max(t[17], 1) / 2.4e3:.2f} us each) + camera-hit shading {t[19] / life:6.3f} "
              f"({t[21]:.3g} passes, {t[20] / max(t[21], 1):.1f} lanes each)")


def main():
    if sys.argv[1] == "--phases":
        return phases(sys.argv[2])
    if sys.argv[1] == "--regen":
        return regen(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
    raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 6)
    at = (raw[:, 2] >> np.uint64(32)).astype(np.int64)  # (px << 16 | py) of the wave's longest tile
    raw[:, 2] &= np.uint64(0xffffffff)
    wit = (raw[:, 5] >> np.uint64(32)).astype(np.int64)  # the wave's own loop iterations in that tile
    raw[:, 5] &= np.uint64(0xffffffff)
    a = raw.astype(np.float64)
    # frames are appended one after another; a frame's records start where the start clock jumps back
    n = len(a)
    starts = a[:, 0]
    valid = starts > 0
    # split into frames by equal sizes (every frame uses the same grid)
    per = int(sys.argv[2]) if len(sys.argv) > 2 else None
    if per is None:
        for cand in range(1, n + 1):
            if n % cand == 0 and cand >= 256 and np.all(np.diff(starts[:cand][valid[:cand]]) < 1e7):
                per = cand
        per = per or n
    for f in range(n // per):
        r = a[f * per:(f + 1) * per]
        rat = at[f * per:(f + 1) * per][r[:, 0] > 0]
        rwit = wit[f * per:(f + 1) * per][r[:, 0] > 0]
        r = r[r[:, 0] > 0]
        t0, t1 = r[:, 0].min(), r[:, 1].max()
        life = (r[:, 1] - r[:, 0]).mean()
        ends = np.sort(r[:, 1])
        us = lambda x: x / 100.0  # 100 MHz ticks -> us
        print(f"frame {f}: {len(r)} waves, frame {us(t1 - t0):8.1f} us, mean wave life {us(life):8.1f} us "
              f"({life / (t1 - t0):.2f}), start spread {us(r[:, 0].max() - t0):6.1f} us, "
              f"tail (median end -> last end) {us(t1 - np.median(ends)):7.1f} us, "
              f"last 1% of waves {us(t1 - ends[int(0.99 * len(ends))]):6.1f} us, "
              f"tiles/wave {r[:, 2].mean():.1f}, longest tile {us(r[:, 3].max()):7.1f} us")
        top = np.argsort(-r[:, 3])[:5]
        print("   longest tiles (px, py of the tile corner: us, most node / leaf iterations of a lane,"
              " the wave's loop iterations):",
              ", ".join(f"({rat[k] >> 16}, {rat[k] & 0xffff}): {us(r[k, 3]):.0f} us {r[k, 4]:.0f}/{r[k, 5]:.0f}"
                        f" wave {rwit[k]}" for k in top))


if __name__ == "__main__":
    main()
