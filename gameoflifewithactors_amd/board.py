"""Board: the GPU engine that replaces the reference's dictionary of cell actors.

Reference seam: ``cells : IDictionary<int*int, CellRef>`` built from ``createCell`` in
``GameOfLife/GameOfLife/GameOfLifeDriver.fs:16-30`` (Akka: ``GameofLife.fs:148-163``).  One ``Board``
holds the whole grid in HBM (bit-packed when the width is a multiple of 32) and ``step(1)`` is one
``updateView()`` tick (``GameOfLifeDriver.fs:32-34``) -- computed by the HIP kernels in
``csrc/`` (streaming pass ``gol_step.hip``) through the C ABI in ``include/gol/gol.h``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib, patterns
from ._lib import BOUNDED, INIT_DOTNET_MOD2, INIT_DOTNET_NEXT2, TORUS, check

__all__ = ["Board", "TORUS", "BOUNDED", "INIT_DOTNET_MOD2", "INIT_DOTNET_NEXT2", "hash_finalize"]


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def hash_finalize(partial_sum: int, width: int, height: int) -> int:
    return int(_lib.load().gol_hash_finalize(partial_sum & 0xFFFFFFFFFFFFFFFF, width, height))


class Board:
    """A width x height Life board on the current HIP device.

    boundary: ``TORUS`` (the actors' topology, GameOfLifeDriver.fs:25) or ``BOUNDED`` (Script.fsx:11).
    tblock_k: upper bound on the generations fused per kernel pass (0 = library default).
    num_gpus: N > 1 spreads the board over devices 0..N-1 of this process as row strips with peer-copied
              halo rows (``gol_create``; bit-identical to one GPU; option {"transport": 2} moves them by RCCL).
    devices: explicit strip placement (``gol_create_multi``), e.g. ``[0, 0, 0]`` runs three strips on one GPU.
    ilv: packed layout, words per interleaved block (0 = library default for the width; 1, 2, 4).
    options: {name: value} passed to gol_set_option after creation (e.g. {"coop": 0}).
    """

    def __init__(self, width: int, height: int, boundary: int = TORUS, tblock_k: int = 0, num_gpus: int = 1,
                 ilv: int = 0, devices=None, options: dict | None = None):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        if devices is not None:
            devs = (ctypes.c_int * len(devices))(*devices)
            check(self._lib.gol_create_multi(width, height, boundary, devs, len(devices), tblock_k, ilv,
                                             ctypes.byref(h)), "gol_create_multi")
        else:
            check(self._lib.gol_create_ex(width, height, boundary, num_gpus, tblock_k, ilv, ctypes.byref(h)),
                  "gol_create")
        self._h = h
        _lib.hold(self)
        self.width, self.height, self.boundary = width, height, boundary
        try:
            for name, value in (options or {}).items():
                self.set_option(name, value)
        except Exception:
            self.close()
            raise

    # ---------------------------------------------------------------- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            check(self._lib.gol_destroy(self._h), "gol_destroy")
            self._h = None
            _lib.release(self)

    def __enter__(self) -> "Board":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- I/O
    def set_cells(self, cells) -> "Board":
        a = np.ascontiguousarray(np.asarray(cells, dtype=np.uint8)).reshape(-1)
        check(self._lib.gol_set_cells(self._h, _u8p(a), a.size), "gol_set_cells")
        return self

    def get_cells(self) -> np.ndarray:
        out = np.empty((self.height, self.width), dtype=np.uint8)
        check(self._lib.gol_get_cells(self._h, _u8p(out), out.size), "gol_get_cells")
        return out

    def get_region(self, x: int, y: int, w: int, h: int) -> np.ndarray:
        """Window of the board as a (h, w) uint8 array (must lie inside the board)."""
        out = np.empty((h, w), dtype=np.uint8)
        check(self._lib.gol_get_region(self._h, x, y, w, h, _u8p(out)), "gol_get_region")
        return out

    def render_gray8(self, alive_value: int = 128, stride: int | None = None) -> np.ndarray:
        """Gray8 frame, pixels[x + y*stride] (GameOfLifeUI.fs:24-28: 128 for actors, 255 for Script.fsx)."""
        stride = self.width if stride is None else stride
        out = np.empty(stride * self.height, dtype=np.uint8)
        check(self._lib.gol_render_gray8(self._h, _u8p(out), stride, alive_value), "gol_render_gray8")
        return out

    # ---------------------------------------------------------------- seeding
    def seed_dotnet(self, seed: int, mode: int = INIT_DOTNET_MOD2) -> "Board":
        check(self._lib.gol_seed_dotnet(self._h, seed, mode), "gol_seed_dotnet")
        return self

    # ---------------------------------------------------------------- snapshots and patterns
    def save_packed(self) -> np.ndarray:
        """Canonical bit-packed snapshot (gol_save_packed): (height, ceil(width/64)) uint64."""
        nc = (self.width + 63) // 64
        out = np.empty((self.height, nc), dtype="<u8")
        check(self._lib.gol_save_packed(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), out.size),
              "gol_save_packed")
        return out

    def load_packed(self, words) -> "Board":
        a = np.ascontiguousarray(np.asarray(words, dtype="<u8")).reshape(-1)
        check(self._lib.gol_load_packed(self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), a.size),
              "gol_load_packed")
        return self

    def save(self, path: str) -> None:
        """Write a snapshot file (patterns.write_snapshot): header + canonical rows, 1 bit per cell."""
        patterns.write_snapshot(path, self.save_packed(), self.width, self.height, self.boundary, self.generation,
                                self.hash())

    @classmethod
    def from_snapshot(cls, path: str, **kw) -> "Board":
        """A new board holding a snapshot file's cells (same size and boundary); the canonical hash recorded
        in the file is checked after the upload.  kw: tblock_k, num_gpus, ilv, devices."""
        head, words = patterns.read_snapshot(path)
        b = cls(head["width"], head["height"], head["boundary"], **kw)
        b.load_packed(words)
        if b.hash() != head["hash"]:
            b.close()
            raise ValueError(f"{path}: board hash after load differs from the snapshot's")
        return b

    def to_rle(self) -> str:
        """The board as RLE text (patterns.to_rle); place it back with place_rle(text, 0, 0)."""
        return patterns.to_rle(self.get_cells())

    def seed_splitmix(self, seed: int) -> "Board":
        check(self._lib.gol_seed_splitmix(self._h, seed & 0xFFFFFFFFFFFFFFFF), "gol_seed_splitmix")
        return self

    def place_rle(self, rle: str, x: int, y: int) -> "Board":
        check(self._lib.gol_place_rle(self._h, rle.encode(), x, y), "gol_place_rle")
        return self

    def clear(self) -> "Board":
        check(self._lib.gol_clear(self._h), "gol_clear")
        return self

    # ---------------------------------------------------------------- options
    def set_option(self, name: str, value: int) -> "Board":
        """Per-board path / tuning option (gol_set_option, include/gol/gol.h lists the names).  The test and A/B
        knobs of csrc/gol_debug.h (_lib.DEBUG_OPTIONS) go to gol_debug_set_option."""
        fn = "gol_debug_set_option" if name in _lib.DEBUG_OPTIONS else "gol_set_option"
        check(getattr(self._lib, fn)(self._h, name.encode(), int(value)), f"{fn}({name})")
        return self

    def get_option(self, name: str) -> int:
        fn = "gol_debug_get_option" if name in _lib.DEBUG_OPTIONS else "gol_get_option"
        v = ctypes.c_int64()
        check(getattr(self._lib, fn)(self._h, name.encode(), ctypes.byref(v)), f"{fn}({name})")
        return v.value

    # ---------------------------------------------------------------- stepping
    def step(self, generations: int = 1) -> "Board":
        check(self._lib.gol_step(self._h, generations), "gol_step")
        return self

    def step_timed(self, generations: int) -> float:
        """gol_step between HIP timing events on the board's stream, synchronised (gol_step_timed): the call's device
        time in microseconds, measured by the HIP runtime the library itself runs on."""
        us = ctypes.c_double()
        check(self._lib.gol_step_timed(self._h, generations, ctypes.byref(us)), "gol_step_timed")
        return us.value

    def synchronize(self) -> None:
        check(self._lib.gol_synchronize(self._h), "gol_synchronize")

    @property
    def generation(self) -> int:
        v = ctypes.c_int64()
        check(self._lib.gol_generation(self._h, ctypes.byref(v)), "gol_generation")
        return v.value

    # ---------------------------------------------------------------- observables
    def population(self) -> int:
        v = ctypes.c_int64()
        check(self._lib.gol_population(self._h, ctypes.byref(v)), "gol_population")
        return v.value

    def hash(self) -> int:
        v = ctypes.c_uint64()
        check(self._lib.gol_hash(self._h, ctypes.byref(v)), "gol_hash")
        return v.value

    def info(self) -> dict:
        w, h = ctypes.c_int64(), ctypes.c_int64()
        b, k, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._lib.gol_info(self._h, *(ctypes.byref(x) for x in (w, h, b, k, p))), "gol_info")
        ilv, pitch = ctypes.c_int(), ctypes.c_int64()
        check(self._lib.gol_layout(self._h, ctypes.byref(ilv), ctypes.byref(pitch)), "gol_layout")
        return {"width": w.value, "height": h.value, "boundary": b.value, "tblock_k": k.value, "packed": bool(p.value),
                "ilv": ilv.value, "pitch": pitch.value}

    @property
    def stream(self) -> int:
        """The hipStream_t the board's kernels are launched on (as an integer handle)."""
        s = ctypes.c_void_p()
        check(self._lib.gol_stream(self._h, ctypes.byref(s)), "gol_stream")
        return s.value or 0

    def parts(self) -> list:
        """Row strips of the board: [{"device", "y0", "rows", "ghost"}] (one entry for a single board)."""
        n = ctypes.c_int()
        check(self._lib.gol_num_parts(self._h, ctypes.byref(n)), "gol_num_parts")
        out = []
        for i in range(n.value):
            d, y0, rows, ghost = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            check(self._lib.gol_part_info(self._h, i, *(ctypes.byref(x) for x in (d, y0, rows, ghost))),
                  "gol_part_info")
            out.append({"device": d.value, "y0": y0.value, "rows": rows.value, "ghost": ghost.value})
        return out

    def transport(self) -> str:
        """How the halo rows move (gol_transport): 'rccl: ...', 'peer: ...' or 'none: ...' with the reason."""
        t = ctypes.c_int()
        note = ctypes.create_string_buffer(512)
        check(self._lib.gol_transport(self._h, ctypes.byref(t), note, len(note)), "gol_transport")
        return {0: "none", 1: "peer", 2: "rccl"}[t.value] + ": " + note.value.decode(errors="replace")

    def pass_timing(self) -> list:
        """Advance one pass of the board's temporal depth with HIP timing events (gol_pass_timing); per row
        strip, microseconds from the pass start to the interior launch's end, to the edge-band stream's
        release (the halo rows landed: the edge-band wait) and to the edge bands' end."""
        n = ctypes.c_int()
        check(self._lib.gol_num_parts(self._h, ctypes.byref(n)), "gol_num_parts")
        arrs = [(ctypes.c_double * n.value)() for _ in range(3)]
        check(self._lib.gol_pass_timing(self._h, n.value, *arrs), "gol_pass_timing")
        return [{"interior_us": round(arrs[0][i], 2), "edge_wait_us": round(arrs[1][i], 2),
                 "edge_done_us": round(arrs[2][i], 2)} for i in range(n.value)]
