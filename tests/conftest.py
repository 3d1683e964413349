import os
import sys
from pathlib import Path

# hardware queues for the renderer's frames in flight, before anything initialises HIP
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import opengl_ray_tracing_amd  # noqa: E402,F401

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpt.so on the GPU)")
    config.addinivalue_line("markers", "slow: longer CPU test")
    config.addinivalue_line("markers", "perf: wall-clock assertion, run only with PT_PERF_TESTS=1")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build libpt.so / liboracle.so in-tree if missing (hipcc cross-compiles without a GPU)."""
    from opengl_ray_tracing_amd import _build
    if not _build.LIB.exists():
        _build.build_native()
    if not _build.ORACLE_LIB.exists():
        _build.build_oracle()
    if not _build.ABI_CALLER.exists():
        _build.build_abi_caller()
    yield
