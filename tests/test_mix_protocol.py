"""The tile mix protocol of the frame kernels (pt_kernels.hip completeItem).

Frames in flight update the running mean (ImportanceSampling_LowDiscrepancySequence/shaders/
pass1.fsh:868-871) inside their kernels, tile by tile, in frame order, without any wave
waiting for another: a frame's last item of a tile mixes the tile if every earlier frame is
mixed into it, and a mixer hands on to later frames that already completed the tile. This
compiles tests/native/mix_protocol_check.cpp -- the same sequentially consistent operations
over std::atomic, 8 threads on shuffled, randomly split items of 9 frames at a time -- and
requires every frame mixed into every tile exactly once and the running mean bit for bit
equal to mixing the frames one after another. The GPU tests (test_gpu_parity.py pipelined /
shared-work frames) check the kernel itself against serial frames."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_tile_mix_protocol_equals_serial_mixing(tmp_path):
    exe = tmp_path / "mix_protocol_check"
    subprocess.run(["g++", "-O2", "-pthread", "-std=c++17", "-ffp-contract=off",
                    str(ROOT / "tests" / "native" / "mix_protocol_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
    _, mixes, handoffs = out.stdout.split()
    assert int(mixes) > 0 and int(handoffs) > 0  # later frames were mixed by an earlier frame's completer
