"""A CPU strip engine built from the ORACLE -- test infrastructure only.

It lets the multi-process strip protocol (gameoflifewithactors_amd/strips.py: partitioning, ghost rows,
DistExchange over gloo, global hash reduction) run on CPU with world_size > 1, so the N > 1 path is
covered without GPUs.  It implements the same engine interface as strips.HipEngine on int32 CPU
tensors holding the same bit-packed strip layout (include/gol/gol.h, gol_strip).
"""
from __future__ import annotations

import numpy as np
import torch

import gol_oracle as o


def _cell_of_bit(width: int, ilv: int) -> np.ndarray:
    """For every stored bit position p = 32*w + b of a row: the cell it holds (include/gol/gol.h layout:
    block k of ilv words, word j bit b = cell 32*ilv*k + j + ilv*b)."""
    p = np.arange(width)
    w, b = p // 32, p % 32
    return (w // ilv) * 32 * ilv + (w % ilv) + ilv * b


def _unpack(words: np.ndarray, width: int, ilv: int = 1) -> np.ndarray:
    """(rows, pitch) int32 -> (rows, width) uint8 cells."""
    bits = np.unpackbits(words.astype("<u4").view(np.uint8), axis=1, bitorder="little")[:, :width]
    out = np.empty_like(bits)
    out[:, _cell_of_bit(width, ilv)] = bits
    return out


def _pack(cells: np.ndarray, pitch: int, ilv: int = 1) -> np.ndarray:
    rows, width = cells.shape
    padded = np.zeros((rows, pitch * 32), np.uint8)
    padded[:, :width] = cells[:, _cell_of_bit(width, ilv)]
    return np.packbits(padded, axis=1, bitorder="little").view("<u4").astype(np.uint32).view(np.int32)


class OracleEngine:
    def __init__(self, device=None, ilv: int = 1):
        self.device = torch.device("cpu")
        self.ilv = ilv

    def ilv_for(self, width, rows=None, boundary=0):
        return self.ilv

    def alloc(self, geom, stream=None):
        return torch.zeros((geom.buffer_rows, geom.pitch), dtype=torch.int32)

    def step(self, geom, src, dst, k, out_begin, out_end, stream=None, spare_waves=0):
        if out_begin >= out_end:
            return
        g = geom.ghost
        lo, hi = out_begin - k, out_end + k
        if geom.boundary == o.BOUNDED:  # rows beyond the board edge are dead: leave them out of the array
            lo, hi = max(lo, -geom.y0), min(hi, geom.height - geom.y0)
            # the oracle needs >= 3 rows: widen on a side that is not the board edge (rows beyond the
            # k-row cone only pollute rows that are discarded)
            while hi - lo < 3:
                if hi < min(geom.rows + g, geom.height - geom.y0):
                    hi += 1
                else:
                    lo -= 1
        if geom.wrap_rows:
            rows = np.arange(lo, hi) % geom.rows
            words = src.numpy()[rows]
        else:
            words = src.numpy()[lo + g:hi + g]
        cells = _unpack(words, geom.width, geom.ilv)
        # torus in x is exact; the array's y edges that are not board edges only pollute rows inside
        # the k-row light cone that is discarded below
        res = o.c_run(cells, k, geom.boundary)
        out = res[out_begin - lo:out_end - lo]
        dst.numpy()[out_begin + g:out_end + g] = _pack(out, geom.pitch, geom.ilv)

    def seed_splitmix(self, geom, buf, seed, stream=None):
        full = o.seed_splitmix(geom.width, geom.height, seed)
        buf.numpy()[geom.ghost:geom.ghost + geom.rows] = _pack(full[geom.y0:geom.y0 + geom.rows], geom.pitch, geom.ilv)

    def set_cells(self, geom, buf, cells_u8, stream=None):
        buf.numpy()[geom.ghost:geom.ghost + geom.rows] = _pack(np.asarray(cells_u8, np.uint8), geom.pitch, geom.ilv)

    def get_cells(self, geom, buf, stream=None):
        return torch.from_numpy(_unpack(buf.numpy()[geom.ghost:geom.ghost + geom.rows], geom.width, geom.ilv))

    def reduce(self, geom, buf, what, stream=None):
        cells = _unpack(buf.numpy()[geom.ghost:geom.ghost + geom.rows], geom.width, geom.ilv)
        if what != "hash":
            return torch.tensor([int(cells.sum())], dtype=torch.int64)
        nc = (geom.width + 63) // 64
        padded = np.zeros((geom.rows, nc * 64), np.uint8)
        padded[:, :geom.width] = cells
        v = np.packbits(padded.reshape(geom.rows, nc, 64), axis=2, bitorder="little").view("<u8")
        v = v.reshape(geom.rows, nc).astype(np.uint64)
        key = (np.arange(geom.rows, dtype=np.uint64)[:, None] + np.uint64(geom.y0)) * np.uint64(nc) + np.arange(
            nc, dtype=np.uint64)[None, :]
        with np.errstate(over="ignore"):
            acc = np.sum(o._fmix64(v ^ o._fmix64(key + np.uint64(0x9E3779B97F4A7C15))), dtype=np.uint64)
        return torch.tensor([int(acc)], dtype=torch.uint64).view(torch.int64)
