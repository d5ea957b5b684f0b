"""Pattern and snapshot formats on either side of the hot path (init / pattern I/O).

* RLE export (``to_rle``): the standard Life run-length format that ``gol_place_rle`` reads, so a board
  region can be written out and placed back.  The reference seeds only from ``System.Random``
  (``GameOfLifeDriver.fs:9-19``); RLE is the interchange format for the pattern configs (BASELINE config 5).
* Board snapshots (``write_snapshot`` / ``read_snapshot``): a small header plus the canonical bit-packed
  rows of ``gol_save_packed`` (row y = ceil(W/64) little-endian uint64, bit i of word j = cell 64j + i).
  Independent of the GPU layout and GPU count, 1 bit per cell, and checked by the canonical hash on load.

Pure host code (numpy); the Board methods in ``board.py`` move the words to and from HBM.
"""
from __future__ import annotations

import struct

import numpy as np

# BASELINE config 5's seeds: the Gosper glider gun (36 cells, period 30) and the R-pentomino
GOSPER_GUN = ("24bo$22bobo$12b2o6b2o12b2o$11bo3bo4b2o12b2o$2o8bo5bo3b2o$2o8bo3bob2o4bobo$10bo5bo7bo$11bo3bo$"
              "12b2o!")
R_PENTOMINO = "b2o$2o$bo!"
NAMED = {"gosper-gun": GOSPER_GUN, "r-pentomino": R_PENTOMINO}


def parse_placements(spec: str) -> list:
    """'NAME_OR_FILE[@x,y]+...' -> [(rle text, x, y)]: a named pattern (gosper-gun, r-pentomino) or an RLE file,
    its top-left at (x, y) (default 0, 0)."""
    out = []
    for part in spec.split("+"):
        what, _, at = part.partition("@")
        x, y = (int(v) for v in at.split(",")) if at else (0, 0)
        if what in NAMED:
            text = NAMED[what]
        else:
            with open(what) as f:
                text = f.read()
        out.append((text, x, y))
    return out


MAGIC = b"GOLSNAP1"
_HEADER = struct.Struct("<8sqqiiqQ")  # magic, width, height, boundary, reserved, generation, hash


def to_rle(cells: np.ndarray, rule: str = "B3/S23", line: int = 70) -> str:
    """RLE text of a (height, width) 0/1 array: ``b`` dead, ``o`` alive, ``$`` end of row, ``!`` end;
    trailing dead cells of a row and trailing empty rows are omitted, lines wrap at `line` characters."""
    cells = np.asarray(cells)
    h, w = cells.shape
    tokens: list[str] = []
    pending_rows = 0  # row ends not yet written (runs of empty rows collapse into "n$")

    def run(n: int, t: str) -> None:
        tokens.append((str(n) if n > 1 else "") + t)

    for y in range(h):
        row = cells[y] != 0
        nz = np.flatnonzero(row)
        if nz.size == 0:
            pending_rows += 1
            continue
        ends_of_rows = pending_rows + (1 if tokens else 0)  # the previous written row's end + empty rows
        if ends_of_rows:
            run(ends_of_rows, "$")
        pending_rows = 0
        r = row[: nz[-1] + 1].astype(np.int8)
        edges = np.flatnonzero(np.diff(r)) + 1
        starts = np.concatenate(([0], edges))
        ends = np.concatenate((edges, [r.size]))
        for s, e in zip(starts, ends):
            run(int(e - s), "o" if r[s] else "b")
    out, cur = [f"x = {w}, y = {h}, rule = {rule}"], ""
    for t in tokens + ["!"]:
        if len(cur) + len(t) > line:
            out.append(cur)
            cur = ""
        cur += t
    out.append(cur)
    return "\n".join(out) + "\n"


def write_snapshot(path: str, words: np.ndarray, width: int, height: int, boundary: int, generation: int,
                   board_hash: int) -> None:
    words = np.ascontiguousarray(words, dtype="<u8")
    if words.size != height * ((width + 63) // 64):
        raise ValueError("snapshot words must be height * ceil(width/64)")
    with open(path, "wb") as f:
        f.write(_HEADER.pack(MAGIC, width, height, boundary, 0, generation, board_hash & 0xFFFFFFFFFFFFFFFF))
        f.write(words.tobytes())


def read_snapshot(path: str) -> tuple[dict, np.ndarray]:
    """(header dict, words) of a snapshot file; raises ValueError on a bad magic or size."""
    with open(path, "rb") as f:
        head = f.read(_HEADER.size)
        if len(head) != _HEADER.size:
            raise ValueError("truncated snapshot header")
        magic, w, h, boundary, _, gen, hsh = _HEADER.unpack(head)
        if magic != MAGIC:
            raise ValueError("not a board snapshot (bad magic)")
        n = h * ((w + 63) // 64)
        words = np.frombuffer(f.read(8 * n), dtype="<u8")
        if words.size != n:
            raise ValueError("truncated snapshot body")
    return {"width": w, "height": h, "boundary": boundary, "generation": gen, "hash": hsh}, words.copy()
