"""Shared test setup.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu`` on the GPU box); everything else runs on
CPU.  The CPU oracle (``oracle/``) is test infrastructure: tests use it only as the checker.
"""
import os
import subprocess
import sys

import pytest

# torch first: it brings its own HIP runtime, which libgol_hip.so then shares (gameoflifewithactors_amd/_lib.py
# _torch_runtime_first); loading the library first would make a later `import torch` fail by design
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
for p in (ROOT, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    """The numpy oracle twin, with the C restatement built (make -C oracle)."""
    if not os.path.exists(os.path.join(ORACLE, "build", "libgol_oracle.so")) or not os.path.exists(
        os.path.join(ORACLE, "build", "actor_protocol")
    ):
        subprocess.run(["make", "-C", ORACLE], check=True, stdout=subprocess.DEVNULL)
    import gol_oracle

    return gol_oracle


@pytest.fixture(autouse=True)
def _bounds_check_build(request):
    """Diagnostic builds only (GOL_LIB=<a library built with -DGOL_CHECK_BOUNDS=1>): after every test, fail it if any
    kernel built a buffer descriptor reaching outside its buffer (gol_debug_bounds).  The shipped library has no such
    symbol and this does nothing."""
    yield
    if "gpu" not in request.keywords or "GOL_LIB" not in os.environ:
        return
    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    fn = getattr(lib, "gol_debug_bounds", None)
    if fn is None:
        return
    fn.restype = __import__("ctypes").c_uint
    bits = fn()
    assert bits == 0, f"out-of-buffer descriptor in this test: tag bits {bits:#x} (gol_step.hip checked_rsrc tags)"
