#!/usr/bin/env python3
"""Concurrency of the frame kernels in a rocprofv3 kernel trace (tools/gpu_shard_trace.sh):
over the last `frames` frame kernels, how many were running at once, the gaps between a
slot's consecutive frames, and each kernel kind's mean duration.

    python tools/trace_overlap.py gpurun_out/strace_c2_8/kernel_trace.csv [frames]
"""
import csv
import sys
from collections import defaultdict

import numpy as np


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    k = [(r["Kernel_Name"], int(r["Queue_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    k.sort(key=lambda x: x[2])
    frame = [x for x in k if "regenKernel" in x[0] or "renderKernel" in x[0]][-frames:]
    t0, t1 = frame[0][2], frame[-1][3]
    win = [x for x in k if x[2] >= t0 and x[3] <= t1]
    print(f"window {1e-3 * (t1 - t0):.1f} us for {frames} frame kernels: {1e-3 * (t1 - t0) / frames:.1f} us per frame")
    by = defaultdict(list)
    for name, q, s, e in win:
        by[name.split("(")[0][:60]].append(e - s)
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        d = np.array(d) * 1e-3
        print(f"  {n:60s} n={len(d):4d} mean {d.mean():8.1f} us  min {d.min():7.1f}  max {d.max():8.1f}  sum/frame {d.sum() / frames:7.1f}")
    # concurrency of frame kernels over time
    ev = sorted([(s, 1) for _, _, s, _ in frame] + [(e, -1) for _, _, _, e in frame])
    cur, last, acc = 0, ev[0][0], defaultdict(float)
    for t, d in ev:
        acc[cur] += t - last
        cur += d
        last = t
    tot = sum(acc.values())
    print("  frame kernels running at once (share of the window):",
          ", ".join(f"{c}: {acc[c] / tot:.2f}" for c in sorted(acc)))
    # any kernel running at all
    ev = sorted([(s, 1) for _, _, s, _ in win] + [(e, -1) for _, _, _, e in win])
    cur, last, idle = 0, ev[0][0], 0
    for t, d in ev:
        if cur == 0:
            idle += t - last
        cur += d
        last = t
    print(f"  no kernel running: {idle / tot:.3f} of the window")
    qs = defaultdict(list)
    for name, q, s, e in frame:
        qs[q].append((s, e))
    gaps = [b[0] - a[1] for v in qs.values() for a, b in zip(v, v[1:])]
    print(f"  frame-kernel queues {len(qs)}; gap between a queue's consecutive frames: mean "
          f"{1e-3 * np.mean(gaps):.1f} us, median {1e-3 * np.median(gaps):.1f}")


if __name__ == "__main__":
    main()
