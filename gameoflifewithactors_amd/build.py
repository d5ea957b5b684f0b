"""Build recipe for libgol_hip.so (gfx950) -- explicit hipcc, in-tree, no JIT cache.

``python -m gameoflifewithactors_amd.build`` or ``__graft_entry__.build()``.  The shared library lands
next to this file so it travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgol_hip.so")
SOURCES = [os.path.join(CSRC, f) for f in ("gol_step.hip", "gol_formats.hip", "gol_resident.hip", "gol_wave.hip", "gol_coop.hip", "gol_lanes.hip", "gol_pipe.hip", "gol_capi.cpp", "gol_multi.cpp")]
HEADERS = [
    os.path.join(CSRC, "gol_bitlogic.h"),
    os.path.join(CSRC, "gol_layout.h"),
    os.path.join(CSRC, "gol_internal.h"),
    os.path.join(CSRC, "gol_multi.h"),
    os.path.join(CSRC, "gol_debug.h"),
    os.path.join(ROOT, "include", "gol", "gol.h"),
]
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    return "hipcc"


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, lib: str = LIB, defines: tuple = (),
          step_src: str | None = None, flags: tuple = (), alt: dict | None = None) -> str:
    """Compile SOURCES for gfx950 into `lib`.  `defines` (e.g. ("GOL_XLANE=0",)), `step_src` (another revision
    of gol_step.hip) and `alt` ({basename: path} of other revisions of any source) build A/B variants for
    experiments."""
    sources = [step_src or SOURCES[0]] + SOURCES[1:]
    if alt:
        sources = [alt.get(os.path.basename(x), x) for x in sources]
    deps = sources + HEADERS + [os.path.abspath(__file__)]
    if not force and not _stale(lib, deps):
        return lib
    objs = []
    tag = "_".join(d.replace("=", "") for d in defines) + ("_alt" if step_src or alt else "") + ("_fl" if flags else "")
    # A/B variants' objects and libraries stay under build/ (git-ignored), not beside the shipped sources
    objdir = os.path.join(ROOT, "build", "obj") if tag else CSRC
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(os.path.abspath(lib)), exist_ok=True)
    procs = []
    for src in sources:  # compile the translation units in parallel (gol_step.hip dominates)
        obj = os.path.join(objdir, os.path.basename(src) + (f".{tag}" if tag else "") + ".o")
        cmd = [
            _hipcc(),
            f"--offload-arch={ARCH}",
            "-O3",
            "-std=c++17",
            "-fPIC",
            "-Wall",
            "-x",
            "hip",
            "-I",
            os.path.join(ROOT, "include"),
            "-I",
            CSRC,
            "-c",
            src,
            "-o",
            obj,
        ] + [f"-D{d}" for d in defines] + list(flags)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return lib


HOST_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "test_host_driver.cpp")
HOST_TEST_EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_host_driver")


def build_host_tests(verbose: bool = True) -> str:
    """Compile the native host-mirror test (tests/cpp/test_host_driver.cpp: include/gol/gol_host.hpp over
    libgol_hip.so, checked against the CPU oracle object oracle/build/gol_oracle.o -- test infrastructure)."""
    oracle_obj = os.path.join(ROOT, "oracle", "build", "gol_oracle.o")
    deps = [HOST_TEST_SRC, os.path.join(ROOT, "include", "gol", "gol_host.hpp"), os.path.join(ROOT, "include", "gol", "gol.h"),
            LIB, oracle_obj]
    if not _stale(HOST_TEST_EXE, deps):
        return HOST_TEST_EXE
    os.makedirs(os.path.dirname(HOST_TEST_EXE), exist_ok=True)
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-pthread", "-I", os.path.join(ROOT, "include"), HOST_TEST_SRC,
           oracle_obj, "-L", HERE, "-lgol_hip", "-Wl,-rpath,$ORIGIN/../../../gameoflifewithactors_amd", "-o",
           HOST_TEST_EXE]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return HOST_TEST_EXE


if __name__ == "__main__":
    build(force="--force" in sys.argv)
