"""bench.py's N > 1 path as the driver runs it (torch.distributed.run, one process per rank),
rehearsed on the one-GPU box: 2 ranks on device 0 with the gloo backend (staged host copies)
instead of RCCL. It drives broadcast_scene, the screen-tile split in batches of frames per
launch, FrameGather after every batch (--gather accum: the f32 running means; --gather display:
the 8-bit presented frame, the running means gathered once after the run) and the
gather-every-frame leg, and rank 0 prints the one JSON line. Reference frame contract:
ImportanceSampling_LowDiscrepancySequence/main.cpp:659-709 (one display() per frame)."""
import json
import math
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("gather", ["accum", "display"])
def test_bench_two_ranks_print_the_line(gather):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--same-device", "--steps", "4", "--warmup", "1",
           "--no-cpu-baseline", "--no-psnr", "--no-reset", "--gather", gather]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(ROOT),
                         env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["scaling"] == "strong"
    assert d["value"] > 0 and math.isfinite(d["value"]) and d["ms_per_step"] > 0
    c = d["config"]
    assert c["frames_per_gather"] == c["frames_per_launch"] >= 2  # one gather per batch of frames
    assert ("RCCL gather of the " + ("displayed frame" if gather == "display" else "running means")) in c["parallelism"]
    assert c["combined_image_finite"] is True
    assert c["combined_image_filled"] == 1.0  # rank 1's tiles reached rank 0's accumulation
    g = d["gather_every_frame"]
    assert g["frames_per_gather"] == 1 and g["ms_per_step"] > 0 and g["value"] > 0
