#!/usr/bin/env python3
"""Register use of every kernel of one HIP source as hipcc reports it (VGPRs, spills, scratch,
occupancy in waves per SIMD), compiled exactly as _build.py compiles it.

    python tools/kernel_regs.py pt_kernels.hip [extra hipcc flags, e.g. -DPT_X=1] [--filter renderKernel]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from opengl_ray_tracing_amd import _build  # noqa: E402


def main():
    args = sys.argv[1:]
    flt = None
    if "--filter" in args:
        i = args.index("--filter")
        flt = args[i + 1]
        del args[i:i + 2]
    src = _build.CSRC / args[0]
    cmd = [_build.HIPCC, *_build.HIP_FLAGS, f"-I{_build.INCLUDE}", f"-I{_build.CSRC}", *args[1:], "-c", str(src),
           "-o", "/tmp/kernel_regs.o", "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    cur = None
    rows = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"VGPRs Spill|SGPRs Spill): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for c in rows:
        if flt and flt not in c["name"]:
            continue
        print(f"{c.get('VGPRs', '?'):>4} vgpr  spill {c.get('VGPRs Spill', '?'):>4}/{c.get('SGPRs Spill', '?'):>4}  "
              f"scratch {c.get('ScratchSize [bytes/lane]', '?'):>4}  waves {c.get('Occupancy [waves/SIMD]', '?')}  "
              f"{c['name'][:110]}")


if __name__ == "__main__":
    main()
