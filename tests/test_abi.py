"""The C-ABI boundary: libpt.so loads without a GPU and exports every entry point
declared in include/*.h; the oracle library exports its checker API."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from opengl_ray_tracing_amd import _build, _native

ROOT = Path(__file__).resolve().parent.parent
HEADERS = [ROOT / "include" / "pt_abi.h", ROOT / "include" / "pt_scene.h"]


def declared_functions(path: Path):
    text = path.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(pt_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def exported_symbols(lib: Path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_headers_declare_api():
    names = set()
    for h in HEADERS:
        names |= set(declared_functions(h))
    for must in ["pt_create", "pt_upload_scene", "pt_upload_env", "pt_render_frame", "pt_trace_closest",
                 "pt_destroy", "pt_last_error", "pt_scene_build_bvh", "pt_hdr_cache", "pt_hdr_load"]:
        assert must in names


@pytest.mark.parametrize("header", HEADERS, ids=lambda p: p.name)
def test_library_exports_every_declared_symbol(header):
    syms = exported_symbols(_build.LIB)
    missing = [n for n in declared_functions(header) if n not in syms]
    assert not missing, missing


def test_ctypes_signatures_cover_headers():
    declared = set()
    for h in HEADERS:
        declared |= set(declared_functions(h))
    assert declared == set(_native.SIGNATURES), declared ^ set(_native.SIGNATURES)


def test_library_loads_without_gpu():
    lib = _native.load()
    n = C.c_int(-1)
    assert lib.pt_device_count(C.byref(n)) == 0
    assert n.value >= 0


def test_create_reports_errors_instead_of_exiting():
    lib = _native.load()
    cfg = _native.PtConfig()
    cfg.width, cfg.height, cfg.integrator, cfg.tile_world = 0, 0, 0, 1
    h = C.c_void_p()
    assert lib.pt_create(C.byref(h), C.byref(cfg)) == -1  # PT_E_INVALID
    assert b"invalid" in lib.pt_last_error(None)


def test_oracle_exports():
    syms = exported_symbols(_build.ORACLE_LIB)
    for n in ["orc_render_pixels", "orc_trace_closest", "orc_wang_hash", "orc_sobol", "orc_pixel_rng",
              "orc_hdr_cache"]:
        assert n in syms


def test_product_does_not_link_oracle():
    out = subprocess.run(["readelf", "-d", str(_build.LIB)], capture_output=True, text=True, check=True).stdout
    assert "oracle" not in out
    assert "orc_" not in " ".join(exported_symbols(_build.LIB))


def test_compiled_cpp_caller_links_against_the_headers_only():
    """tests/native/abi_caller.cpp -- INTEGRATION.md's DisneyBRDF display() loop and BVH's debug
    ray as a C++ program built with g++ against include/pt_abi.h + pt_scene.h and -lpt -- links
    and loads libpt.so without a GPU (--version calls pt_abi_version only)."""
    exe = _build.build_abi_caller()
    out = subprocess.run([str(exe), "--version"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert int(out.stdout) == _native.load().pt_abi_version()
    need = subprocess.run(["readelf", "-d", str(exe)], capture_output=True, text=True, check=True).stdout
    assert "libpt.so" in need and "oracle" not in need
