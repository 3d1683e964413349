"""In-tree native build: libpt.so (HIP kernels + C-ABI runtime + host scene
prep) for gfx950, and the test-only oracle (oracle/liboracle.so).

The built shared objects stay in the source tree (git-ignored) so they travel
to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
BUILD = PKG / "_objs"
LIB = PKG / "libpt.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle.so"

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = "gfx950"

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    # exact single-rounding float semantics, matching the CPU checker
    "-ffp-contract=off",
    # no SLP packing of the scalar shading/triangle code into v_pk_* pairs: the
    # lane shuffles it needs raised the MIS megakernel to 239 VGPRs (129 -> 167
    # Lambert / 187 MIS without it) and cost 4-6 % per frame on c2/c3/c4
    # (tools/tune.py); visitNode's explicit float2 slab pairs stay packed
    "-fno-slp-vectorize",
    "-Wall", "-Wno-unused-function",
]
CXX_FLAGS = ["-O2", "-fPIC", "-pthread", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-Wall",
             "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include"]

SOURCES = {
    "pt_kernels.o": ("hip", CSRC / "pt_kernels.hip", [CSRC / "pt_device.h", CSRC / "pt_kernels.h", CSRC / "pt_trace.h", INCLUDE / "pt_scene.h",
                                                       INCLUDE / "pt_fmath.h"]),
    "pt_regen.o": ("hip", CSRC / "pt_regen.hip", [CSRC / "pt_device.h", CSRC / "pt_kernels.h", CSRC / "pt_trace.h",
                                                   INCLUDE / "pt_fmath.h"]),
    "pt_envcache.o": ("hip", CSRC / "pt_envcache.hip", [CSRC / "pt_kernels.h"]),
    "pt_primary.o": ("hip", CSRC / "pt_primary.hip", [CSRC / "pt_kernels.h"]),
    "pt_build.o": ("hip", CSRC / "pt_build.hip", [CSRC / "pt_kernels.h"]),
    "pt_runtime.o": ("cxx", CSRC / "pt_runtime.cpp", [CSRC / "pt_kernels.h", INCLUDE / "pt_abi.h", INCLUDE / "pt_scene.h",
                                                       INCLUDE / "pt_fmath.h", CSRC / "pt_rccl.h"]),
    "pt_rccl.o": ("cxx", CSRC / "pt_rccl.cpp", [CSRC / "pt_rccl.h"]),
    "scene.o": ("cxx", CSRC / "scene.cpp", [INCLUDE / "pt_scene.h"]),
}


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
    return r


def build_native(force: bool = False, verbose: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    jobs = []
    objs = []
    for obj, (kind, src, deps) in SOURCES.items():
        out = BUILD / obj
        objs.append(out)
        if force or _stale(out, [src, *deps]):
            inc = [f"-I{INCLUDE}", f"-I{CSRC}"]
            if kind == "hip":
                cmd = [HIPCC, *HIP_FLAGS, *inc, "-c", str(src), "-o", str(out)]
            else:
                cmd = ["g++", *CXX_FLAGS, *inc, "-c", str(src), "-o", str(out)]
            jobs.append(cmd)
    if jobs:
        with ThreadPoolExecutor(max_workers=min(4, len(jobs))) as ex:
            for r in ex.map(_run, jobs):
                if verbose and (r.stdout or r.stderr):
                    sys.stderr.write(r.stdout + r.stderr)
    if force or jobs or _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-pthread", "-o", str(LIB), *map(str, objs), "-ldl"])
    return LIB


VARIANTS = PKG / "_variants"


def variant_lib(name: str) -> Path:
    return VARIANTS / f"libpt_{name}.so"


def build_variant(name: str, defines: dict, hip_flags=()) -> Path:
    """A tuning build of libpt.so with extra -D defines (e.g. PT_MIN_WAVES, PT_LDS_STACK)
    and extra hipcc flags, kept in-tree under _variants/ so tools/tune.py can A/B it on
    the GPU box."""
    out_dir = VARIANTS / name
    out_dir.mkdir(parents=True, exist_ok=True)
    dflags = [f"-D{k}={v}" for k, v in defines.items()]
    inc = [f"-I{INCLUDE}", f"-I{CSRC}"]
    objs, cmds = [], []
    for obj, (kind, src, deps) in SOURCES.items():
        out = out_dir / obj
        objs.append(out)
        if kind == "hip":
            cmds.append([HIPCC, *HIP_FLAGS, *hip_flags, *dflags, *inc, "-c", str(src), "-o", str(out)])
        else:
            cmds.append(["g++", *CXX_FLAGS, *dflags, *inc, "-c", str(src), "-o", str(out)])
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(_run, cmds))
    lib = variant_lib(name)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-pthread", "-o", str(lib), *map(str, objs), "-ldl"])
    return lib


ABI_CALLER_SRC = ROOT / "tests" / "native" / "abi_caller.cpp"
ABI_CALLER = ROOT / "tests" / "native" / "abi_caller"


def build_abi_caller(force: bool = False) -> Path:
    """Test infrastructure: the compiled reference-side caller of the C ABI (tests/native/abi_caller.cpp,
    INTEGRATION.md's DisneyBRDF display() loop), g++ against include/*.h and -lpt only."""
    deps = [ABI_CALLER_SRC, INCLUDE / "pt_abi.h", INCLUDE / "pt_scene.h", LIB]
    if force or _stale(ABI_CALLER, deps):
        _run(["g++", "-std=c++17", "-O2", "-Wall", str(ABI_CALLER_SRC), f"-I{INCLUDE}", f"-L{PKG}", "-lpt",
              "-Wl,-rpath,$ORIGIN/../../opengl_ray_tracing_amd", "-o", str(ABI_CALLER)])
    return ABI_CALLER


def build_oracle(force: bool = False) -> Path:
    """Test infrastructure only (see oracle/pt_oracle.h)."""
    src = [ORACLE_DIR / "pt_oracle.c", ORACLE_DIR / "pt_oracle.h", ORACLE_DIR / "Makefile", INCLUDE / "pt_fmath.h"]
    if force or _stale(ORACLE_LIB, src):
        _run(["make", "-s", "-C", str(ORACLE_DIR), "-B" if force else "all"])
    return ORACLE_LIB


if __name__ == "__main__":
    build_native(force="--force" in sys.argv, verbose=True)
    build_oracle(force="--force" in sys.argv)
    build_abi_caller(force="--force" in sys.argv)
    print(LIB)
    print(ORACLE_LIB)
