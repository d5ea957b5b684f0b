"""ctypes binding of libgol_hip.so (the C ABI declared in include/gol/gol.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be loaded this module
raises, and every Board operation goes through the library.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GOL_LIB") or os.path.join(HERE, "libgol_hip.so")  # GOL_LIB: A/B experiments only

GOL_OK = 0
GOL_ERR_INVALID = -1
GOL_ERR_HIP = -2
GOL_ERR_OOM = -3
GOL_ERR_UNSUPPORTED = -4
GOL_ERR_NO_DEVICE = -5

TORUS = 0
BOUNDED = 1
TRANSPORT_NONE, TRANSPORT_PEER, TRANSPORT_RCCL = 0, 1, 2
INIT_DOTNET_MOD2 = 0
INIT_DOTNET_NEXT2 = 1

_ERRORS = {
    GOL_ERR_INVALID: ValueError,
    GOL_ERR_HIP: RuntimeError,
    GOL_ERR_OOM: MemoryError,
    GOL_ERR_UNSUPPORTED: NotImplementedError,
    GOL_ERR_NO_DEVICE: RuntimeError,
}


class GolError(RuntimeError):
    pass


class Xfer(ctypes.Structure):
    """``gol_xfer`` (include/gol/gol.h): one halo message of a multi-part board's pass."""

    _fields_ = [("part", ctypes.c_int32), ("op", ctypes.c_int32), ("peer", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("row", ctypes.c_int64), ("nrows", ctypes.c_int64)]


class Strip(ctypes.Structure):
    """``gol_strip`` (include/gol/gol.h): geometry of one row strip of a (multi-GPU) board."""

    _fields_ = [
        ("width", ctypes.c_int64),
        ("height", ctypes.c_int64),
        ("y0", ctypes.c_int64),
        ("rows", ctypes.c_int64),
        ("ghost", ctypes.c_int64),
        ("pitch", ctypes.c_int64),
        ("boundary", ctypes.c_int32),
        ("wrap_rows", ctypes.c_int32),
        ("ilv", ctypes.c_int32),
        ("spare_waves", ctypes.c_int32),
    ]


_lib = None
# Objects that keep the loaded CDLL and may call it later (open Board handles, strips.HipEngine): unload() refuses
# while any is alive, since a call through a dlclosed library jumps into unmapped code
import weakref  # noqa: E402

_holders: "weakref.WeakSet" = weakref.WeakSet()


def hold(obj) -> None:
    """Register `obj` as a user of the loaded library until release(obj) or its collection."""
    _holders.add(obj)


def release(obj) -> None:
    _holders.discard(obj)


i64 = ctypes.c_int64
u64 = ctypes.c_uint64
vp = ctypes.c_void_p
u8p = ctypes.POINTER(ctypes.c_uint8)
i64p = ctypes.POINTER(ctypes.c_int64)
u64p = ctypes.POINTER(ctypes.c_uint64)
ip = ctypes.POINTER(ctypes.c_int)
sp = ctypes.POINTER(Strip)

# name -> (restype, argtypes).  Must cover every function include/gol/gol.h declares.
SIGNATURES = {
    "gol_create": (ctypes.c_int, [i64, i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]),
    "gol_create_ex": (ctypes.c_int, [i64, i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(vp)]),
    "gol_create_multi": (ctypes.c_int, [i64, i64, ctypes.c_int, ip, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(vp)]),
    "gol_num_parts": (ctypes.c_int, [vp, ip]),
    "gol_part_info": (ctypes.c_int, [vp, ctypes.c_int, ip, i64p, i64p, i64p]),
    "gol_destroy": (ctypes.c_int, [vp]),
    "gol_set_cells": (ctypes.c_int, [vp, u8p, i64]),
    "gol_get_cells": (ctypes.c_int, [vp, u8p, i64]),
    "gol_get_region": (ctypes.c_int, [vp, i64, i64, i64, i64, u8p]),
    "gol_seed_dotnet": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int]),
    "gol_seed_splitmix": (ctypes.c_int, [vp, u64]),
    "gol_save_packed": (ctypes.c_int, [vp, u64p, i64]),
    "gol_load_packed": (ctypes.c_int, [vp, u64p, i64]),
    "gol_place_rle": (ctypes.c_int, [vp, ctypes.c_char_p, i64, i64]),
    "gol_clear": (ctypes.c_int, [vp]),
    "gol_step": (ctypes.c_int, [vp, i64]),
    "gol_generation": (ctypes.c_int, [vp, i64p]),
    "gol_synchronize": (ctypes.c_int, [vp]),
    "gol_render_gray8": (ctypes.c_int, [vp, u8p, i64, ctypes.c_uint8]),
    "gol_population": (ctypes.c_int, [vp, i64p]),
    "gol_hash": (ctypes.c_int, [vp, u64p]),
    "gol_info": (ctypes.c_int, [vp, i64p, i64p, ip, ip, ip]),
    "gol_stream": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
    "gol_pass_timing": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "gol_layout": (ctypes.c_int, [vp, ip, i64p]),
    "gol_default_ilv": (ctypes.c_int, [i64]),
    "gol_default_tblock": (ctypes.c_int, [ctypes.c_int]),
    "gol_supported_k": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "gol_default_layout": (ctypes.c_int, [i64, i64, ctypes.c_int, ip, ip]),
    "gol_last_error": (ctypes.c_char_p, []),
    "gol_version": (ctypes.c_char_p, []),
    "gol_arch_supported": (ctypes.c_int, [ctypes.c_char_p]),
    "gol_strip_step": (ctypes.c_int, [sp, vp, vp, ctypes.c_int, i64, i64, vp]),
    "gol_strip_seed_splitmix": (ctypes.c_int, [sp, vp, u64, vp]),
    "gol_strip_pack": (ctypes.c_int, [sp, vp, vp, vp]),
    "gol_strip_unpack": (ctypes.c_int, [sp, vp, vp, i64, ctypes.c_uint8, vp]),
    "gol_strip_population": (ctypes.c_int, [sp, vp, vp, vp]),
    "gol_strip_hash_partial": (ctypes.c_int, [sp, vp, vp, vp]),
    "gol_hash_finalize": (u64, [u64, i64, i64]),
    "gol_strip_plan": (ctypes.c_int, [sp, ctypes.c_int, i64, i64, i64p, i64p]),
    "gol_strip_plan_ex": (ctypes.c_int, [sp, ctypes.c_int, i64, i64, i64p, i64]),
    "gol_set_option": (ctypes.c_int, [vp, ctypes.c_char_p, i64]),
    "gol_transport": (ctypes.c_int, [vp, ip, ctypes.c_char_p, i64]),
    "gol_exchange_plan": (ctypes.c_int, [i64, ctypes.c_int, ctypes.c_int, i64, ctypes.c_int, ctypes.POINTER(Xfer), i64,
                                         i64p]),
    "gol_get_option": (ctypes.c_int, [vp, ctypes.c_char_p, i64p]),
    "gol_device_count": (ctypes.c_int, [ip]),
    "gol_step_timed": (ctypes.c_int, [vp, i64, ctypes.POINTER(ctypes.c_double)]),
    # test and A/B knobs (csrc/gol_debug.h: internal, not part of the gol.h boundary)
    "gol_debug_set_option": (ctypes.c_int, [vp, ctypes.c_char_p, i64]),
    "gol_debug_get_option": (ctypes.c_int, [vp, ctypes.c_char_p, i64p]),
    "gol_debug_option_names": (ctypes.c_char_p, []),
    "gol_debug_pipe_plan": (ctypes.c_int, [sp, ctypes.c_int, i64, i64, i64, i64p, i64]),
    "gol_debug_pipe_errors": (ctypes.c_int, [ip]),
}

# Names gol_debug_set_option / gol_debug_get_option take (csrc/gol_debug.h); Board.set_option routes them there.
# The library exports its own list (gol_debug_option_names); tests/test_cpu_host.py checks this one against it.
DEBUG_OPTIONS = frozenset({"coop_epoch", "coop_spin_limit", "coop_r", "resident_threads", "coop_launch",
                           "lanes_launches"})


def _elf_sections(data: bytes, base: int = 0):
    """(name, offset, size) of every section of the 64-bit little-endian ELF image at data[base:]."""
    import struct

    shoff, = struct.unpack_from("<Q", data, base + 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, base + 0x3A)

    def sec(i):
        name, _type, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", data, base + shoff + i * shentsize)
        return name, off, size

    _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        name, off, size = sec(i)
        end = data.index(b"\0", base + stroff + name)
        yield data[base + stroff + name:end].decode(errors="replace"), off, size


def device_code_fingerprint(path: str = LIB_PATH, kernel: str = "gol_stream_step") -> str | None:
    """sha256 (first 16 hex digits) of the gfx950 code object that holds `kernel` (the translation unit of the hot
    kernel, csrc/gol_step.hip) inside a built library's `.hip_fatbin`.  PMC measurements (profiles/pmc_traffic.json)
    record it, and bench.py uses a measurement only for the device code it was taken on; edits to the other
    translation units (formats, coop, ...) leave it unchanged."""
    import hashlib
    import struct

    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    if data[:4] != b"\x7fELF" or data[4] != 2:
        return None
    fat = next(((off, size) for name, off, size in _elf_sections(data) if name == ".hip_fatbin"), None)
    if fat is None:
        return None
    blob = data[fat[0]:fat[0] + fat[1]]
    # the device code objects are whole ELF images inside the offload bundles: hash the one(s) naming the kernel
    h = hashlib.sha256()
    found = False
    pos = blob.find(b"\x7fELF")
    while pos >= 0:
        try:
            shoff, = struct.unpack_from("<Q", blob, pos + 0x28)
            shentsize, shnum = struct.unpack_from("<HH", blob, pos + 0x3A)
            size = shoff + shentsize * shnum
        except struct.error:
            break
        image = blob[pos:pos + size]
        if kernel.encode() in image:
            h.update(image)
            found = True
        pos = blob.find(b"\x7fELF", pos + max(size, 4))
    return h.hexdigest()[:16] if found else None


def hip_runtimes() -> list:
    """Paths of every HIP runtime (libamdhip64) mapped into this process (Linux /proc/self/maps)."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and "libamdhip64" in os.path.basename(parts[-1]):
                    paths.add(os.path.realpath(parts[-1]))
    except OSError:
        pass
    return sorted(paths)


def _torch_runtime_first() -> None:
    """torch ships its own HIP runtime (torch/lib/libamdhip64.so, ROCm 7.0) under the same soname as the one
    libgol_hip.so links (/opt/rocm/lib/libamdhip64.so.7, ROCm 7.2), and the dynamic loader binds every later
    library to whichever was loaded first.  If libgol_hip.so came first, torch's own kernels ran on the 7.2
    runtime and its lazy init failed ("No HIP GPUs are available", profiles/r2/pytest_parity_d.log).

    So the rule is: a process that uses torch imports it BEFORE the library (then both share torch's runtime), and a
    process without torch (the F# host, the C++ mirror, bench.py's handle leg) runs on /opt/rocm's.  load() does not
    import torch itself (no torch import as a side effect of loading the library); when torch is
    already imported it is already mapped, and when it is not, an import hook warns at a LATER `import torch` with
    this explanation instead of leaving torch to fail at its first kernel."""
    import sys

    if "torch" in sys.modules:
        return
    sys.meta_path.insert(0, _TorchAfterLibrary())


class _TorchAfterLibrary:
    """sys.meta_path finder installed when libgol_hip.so was loaded without torch: importing torch afterwards binds
    torch to /opt/rocm's HIP runtime, on which torch's own kernels fail ("No HIP GPUs are available").  It warns once,
    at that import, with the reason (a RuntimeWarning rather than an ImportError: a host process that imports torch
    only for bookkeeping keeps working, and the library itself is unaffected)."""

    warned = False

    def find_spec(self, name, path=None, target=None):
        if name == "torch" and not _TorchAfterLibrary.warned and _lib is not None:
            rts = hip_runtimes()
            if len(rts) == 1 and "/torch/" not in rts[0]:
                import warnings

                _TorchAfterLibrary.warned = True
                warnings.warn("torch imported after gameoflifewithactors_amd loaded libgol_hip.so on " + rts[0] +
                              ": torch's kernels cannot run on that HIP runtime; import torch before the library",
                              RuntimeWarning, stacklevel=2)
        return None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libgol_hip.so; raises (never falls back) when it is absent.  Raises GolError when two HIP runtimes end
    up mapped into the process (torch's and /opt/rocm's)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GolError(
            f"{path} not found: build it with `python -m gameoflifewithactors_amd.build` "
            "(there is no CPU fallback for the hot path)"
        )
    lib = ctypes.CDLL(path)
    rts = hip_runtimes()
    if len(rts) > 1:
        raise GolError("two HIP runtimes are mapped into this process (" + ", ".join(rts) + "): torch and "
                       "libgol_hip.so must share one; import torch before loading libgol_hip.so")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    _torch_runtime_first()
    return lib


def unload() -> None:
    """dlclose libgol_hip.so now, while the HIP runtime -- and a profiler attached to it -- is still alive, so its
    device code is unregistered here and not in the process-exit destructors (DESIGN.md 6 "Exit under rocprofv3").
    Close every board first: GolError while any Board or strip engine that holds the library is alive.  load()
    maps it again afterwards."""
    global _lib
    if _lib is None:
        return
    if len(_holders):
        raise GolError(f"unload: {len(_holders)} board(s) / engine(s) still hold libgol_hip.so; close them first")
    import _ctypes

    handle = _lib._handle
    _lib = None
    _ctypes.dlclose(handle)


def device_count() -> int:
    """HIP devices visible to the library (gol_device_count; no torch needed)."""
    n = ctypes.c_int()
    check(load().gol_device_count(ctypes.byref(n)), "gol_device_count")
    return n.value


def exchange_plan(height: int, boundary: int, nparts: int, ghost: int, k: int) -> list:
    """gol_exchange_plan: the halo messages of one pass of a multi-part board, in issue order per part:
    [(part, "send"|"recv", peer, first buffer row, rows)].  Host-only."""
    lib = load()
    n = ctypes.c_int64()
    check(lib.gol_exchange_plan(height, boundary, nparts, ghost, k, None, 0, ctypes.byref(n)), "gol_exchange_plan")
    ops = (Xfer * n.value)()
    check(lib.gol_exchange_plan(height, boundary, nparts, ghost, k, ops, n.value, ctypes.byref(n)), "gol_exchange_plan")
    return [(x.part, "send" if x.op == 0 else "recv", x.peer, x.row, x.nrows) for x in ops]


def check(rc: int, what: str = "") -> None:
    if rc == GOL_OK:
        return
    msg = load().gol_last_error().decode(errors="replace")
    exc = _ERRORS.get(rc, GolError)
    raise exc(f"{what}: {msg} (code {rc})" if what else f"{msg} (code {rc})")
