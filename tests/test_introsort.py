"""pt::exactSort (opengl_ray_tracing_amd/csrc/pt_introsort.h) gives std::sort's permutation.

The reference builders sort tied records with std::sort (OpenglRayTracing/main.cpp:412-418,
467-469, 538-544), so the tree depends on exactly which permutation libstdc++'s introsort
leaves. scene.cpp reproduces it with a parallel restatement of that introsort; this
compiles tests/native/introsort_check.cpp against the header with the same g++ the library
is built with and compares it to std::sort (serial and threaded) and its heapsort fallback
to std::partial_sort, on tie-heavy, presorted, reversed, organ-pipe and adversarial
(McIlroy) inputs up to 2^20 records. The c5 tree digest test (test_ref_pinned.py) checks
the same thing end to end against the reference build."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_exact_sort_equals_std_sort(tmp_path):
    exe = tmp_path / "introsort_check"
    subprocess.run(["g++", "-O2", "-pthread", "-std=c++17", f"-I{ROOT / 'opengl_ray_tracing_amd' / 'csrc'}",
                    str(ROOT / "tests" / "native" / "introsort_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
    assert int(out.stdout.split()[3]) > 0  # the depth-limit heapsort path ran
