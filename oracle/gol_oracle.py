"""CPU ORACLE (numpy twin of gol_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker.  The product package (``gameoflifewithactors_amd``) never imports it.

Restates the reference's hot path (see gol_oracle.c for the full citation list):

* rule      ``GameOfLife/GameOfLife/GameOfLifeLogic.fs:59-63`` (``GameOfLifeAkka/GameofLife.fs:108-112``)
* torus     ``GameOfLifeDriver.fs:21-25``; bounded ``Script.fsx:6-18``
* snapshot  ``GameOfLifeLogic.fs:47-55`` under the Reset->State phase barrier = synchronous step
* init      ``GameOfLifeDriver.fs:9-11,16-19`` (dotnet-mod2), ``Script.fsx:25-27`` (dotnet-next2)
* pixels    ``GameOfLifeUI.fs:24-28`` (128/0), ``Script.fsx:33-35`` (255/0)

PARITY PIN STATUS: the reference ships no tests or fixtures for this path and cannot run here, so
this oracle is pinned by external known answers (tests/test_oracle.py) and by agreement with the
independent C restatement and the actor-protocol restatement; beyond that, "parity unpinned".

Boards are ``numpy.uint8`` arrays of shape ``(H, W)`` indexed ``[y, x]`` -- the same memory order as
the reference's ``pixels[x + y*size]``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

TORUS = 0
BOUNDED = 1

MBIG = 2147483647
MSEED = 161803398

_U64 = np.uint64


def _wrap32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


class DotNetRandom:
    """.NET Framework 4.x ``System.Random(int)`` (Knuth subtractive generator).

    Call sites in the reference: ``GameOfLifeDriver.fs:10-11``, ``GameofLife.fs:141-142``,
    ``Script.fsx:25,27``.  Pinned by published values only (see tests/test_oracle.py).
    """

    def __init__(self, seed: int):
        seed = _wrap32(seed)
        subtraction = MBIG if seed == -(1 << 31) else abs(seed)
        mj = MSEED - subtraction
        mk = 1
        sa = [0] * 56
        sa[55] = mj
        for i in range(1, 55):
            ii = (21 * i) % 55
            sa[ii] = mk
            mk = _wrap32(mj - mk)
            if mk < 0:
                mk += MBIG
            mj = sa[ii]
        for _ in range(1, 5):
            for i in range(1, 56):
                sa[i] = _wrap32(sa[i] - sa[1 + (i + 30) % 55])
                if sa[i] < 0:
                    sa[i] += MBIG
        self._sa = sa
        self._inext = 0
        self._inextp = 21

    def _internal_sample(self) -> int:
        i, j = self._inext + 1, self._inextp + 1
        if i >= 56:
            i = 1
        if j >= 56:
            j = 1
        ret = _wrap32(self._sa[i] - self._sa[j])
        if ret == MBIG:
            ret -= 1
        if ret < 0:
            ret += MBIG
        self._sa[i] = ret
        self._inext, self._inextp = i, j
        return ret

    def next(self, max_value: int | None = None) -> int:
        if max_value is None:
            return self._internal_sample()
        return int(self._internal_sample() * (1.0 / MBIG) * max_value)


def seed_dotnet(width: int, height: int, seed: int, mode: int = 0) -> np.ndarray:
    """mode 0: x outer / y inner, ``Next() % 2 = 0`` (GameOfLifeDriver.fs:9-11,16-19);
    mode 1: ``Array2D.init`` index 0 outer, ``Next 2 = 0`` (Script.fsx:27)."""
    r = DotNetRandom(seed)
    b = np.zeros((height, width), dtype=np.uint8)
    for x in range(width):
        for y in range(height):
            b[y, x] = (r.next() % 2 == 0) if mode == 0 else (r.next(2) == 0)
    return b


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + _U64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
        return z ^ (z >> _U64(31))


def seed_splitmix(width: int, height: int, seed: int) -> np.ndarray:
    """Build-owned large-board init: bit (x & 31) of low32(splitmix64(seed ^ (y*ceil(W/32) + x//32)))."""
    wc = (width + 31) // 32
    chunk = (np.arange(height, dtype=np.uint64)[:, None] * _U64(wc) + np.arange(wc, dtype=np.uint64)[None, :])
    bits = (_splitmix64(chunk ^ _U64(seed & 0xFFFFFFFFFFFFFFFF)) & _U64(0xFFFFFFFF)).astype(np.uint32)
    cells = ((bits[:, :, None] >> np.arange(32, dtype=np.uint32)[None, None, :]) & 1).astype(np.uint8)
    return np.ascontiguousarray(cells.reshape(height, wc * 32)[:, :width])


def neighbour_count(b: np.ndarray, boundary: int) -> np.ndarray:
    """Number of live cells among the 8 neighbours (GameOfLifeDriver.fs:21-25 / Script.fsx:6-13)."""
    h, w = b.shape
    if boundary == TORUS:
        n = np.zeros((h, w), dtype=np.int32)
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if dx or dy:
                    n += np.roll(np.roll(b, -dy, axis=0), -dx, axis=1)
        return n
    p = np.zeros((h + 2, w + 2), dtype=np.int32)
    p[1:-1, 1:-1] = b
    n = np.zeros((h, w), dtype=np.int32)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx or dy:
                n += p[1 + dy : 1 + dy + h, 1 + dx : 1 + dx + w]
    return n


def step(b: np.ndarray, boundary: int = TORUS) -> np.ndarray:
    """One synchronous generation; rule GameOfLifeLogic.fs:59-63 (a>3||a<2 dead, 3 alive, else keep)."""
    h, w = b.shape
    if h < 3 or w < 3:
        raise ValueError("board must be at least 3x3 (smaller tori alias neighbours; see DESIGN.md)")
    a = neighbour_count(b, boundary)
    return np.where(a == 3, 1, np.where(a == 2, b, 0)).astype(np.uint8)


def run(b: np.ndarray, generations: int, boundary: int = TORUS) -> np.ndarray:
    for _ in range(generations):
        b = step(b, boundary)
    return b


def population(b: np.ndarray) -> int:
    return int(np.count_nonzero(b))


def _fmix64(k: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        k = k ^ (k >> _U64(33))
        k = k * _U64(0xFF51AFD7ED558CCD)
        k = k ^ (k >> _U64(33))
        k = k * _U64(0xC4CEB9FE1A85EC53)
        return k ^ (k >> _U64(33))


def board_hash(b: np.ndarray) -> int:
    """Canonical hash: sum_{y,j} fmix64(v ^ fmix64(y*ceil(W/64)+j + phi)), then dims mix."""
    h, w = b.shape
    nc = (w + 63) // 64
    padded = np.zeros((h, nc * 64), dtype=np.uint8)
    padded[:, :w] = b != 0
    v = np.packbits(padded.reshape(h, nc, 64), axis=2, bitorder="little").view("<u8").reshape(h, nc)
    key = np.arange(h * nc, dtype=np.uint64).reshape(h, nc)
    with np.errstate(over="ignore"):
        terms = _fmix64(v.astype(np.uint64) ^ _fmix64(key + _U64(0x9E3779B97F4A7C15)))
        acc = int(np.sum(terms, dtype=np.uint64))
        dims = _fmix64(np.array([(w * 0x100000001B3 + h) & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))
        return int(_fmix64(np.array([acc], dtype=np.uint64) ^ dims)[0])


def render_gray8(b: np.ndarray, alive_value: int = 128, stride: int | None = None) -> np.ndarray:
    """GameOfLifeUI.fs:24-28: pixels[x + y*stride] = alive_value | 0 (flat array)."""
    h, w = b.shape
    stride = w if stride is None else stride
    out = np.zeros(h * stride, dtype=np.uint8)
    out.reshape(h, stride)[:, :w] = np.where(b != 0, alive_value, 0)
    return out


def parse_rle(rle: str) -> list[tuple[int, int]]:
    """Standard Life RLE -> list of live (dx, dy)."""
    cells = []
    lines = [ln for ln in rle.splitlines() if not ln.lstrip().startswith(("#", "x"))]
    body = "".join(lines)
    dx = dy = 0
    count = ""
    for c in body:
        if c.isdigit():
            count += c
            continue
        if c in " \t\r\n":
            continue
        if c == "!":
            break
        n = int(count) if count else 1
        count = ""
        if c == "$":
            dy += n
            dx = 0
        elif c in "b.":
            dx += n
        elif c.isalpha():
            cells.extend((dx + i, dy) for i in range(n))
            dx += n
        else:
            raise ValueError(f"bad RLE token {c!r}")
    return cells


def place_rle(b: np.ndarray, rle: str, x0: int, y0: int) -> np.ndarray:
    h, w = b.shape
    for dx, dy in parse_rle(rle):
        b[(y0 + dy) % h, (x0 + dx) % w] = 1
    return b


GOSPER_GUN = (
    "24bo$22bobo$12b2o6b2o12b2o$11bo3bo4b2o12b2o$2o8bo5bo3b2o$2o8bo3bob2o4bobo$10bo5bo7bo$11bo3bo$12b2o!"
)
R_PENTOMINO = "b2o$2o$bo!"
GLIDER = "bo$2bo$3o!"
BLINKER = "3o!"
BLOCK = "2o$2o!"


# ---------------------------------------------------------------- C restatement (ctypes)
_HERE = os.path.dirname(os.path.abspath(__file__))
_C = None


def c_oracle() -> ctypes.CDLL:
    """Load oracle/build/libgol_oracle.so (built by ``make -C oracle`` / __graft_entry__.build())."""
    global _C
    if _C is None:
        path = os.path.join(_HERE, "build", "libgol_oracle.so")
        lib = ctypes.CDLL(path)
        i64, u8p = ctypes.c_int64, ctypes.POINTER(ctypes.c_uint8)
        lib.oracle_step.argtypes = [u8p, u8p, i64, i64, ctypes.c_int]
        lib.oracle_run.argtypes = [u8p, u8p, i64, i64, ctypes.c_int, i64]
        lib.oracle_hash.argtypes = [u8p, i64, i64]
        lib.oracle_hash.restype = ctypes.c_uint64
        lib.oracle_population.argtypes = [u8p, i64, i64]
        lib.oracle_population.restype = ctypes.c_int64
        lib.oracle_seed_dotnet.argtypes = [u8p, i64, i64, ctypes.c_int32, ctypes.c_int]
        lib.oracle_seed_splitmix.argtypes = [u8p, i64, i64, ctypes.c_uint64]
        lib.oracle_render_gray8.argtypes = [u8p, i64, i64, u8p, i64, ctypes.c_uint8]
        lib.oracle_place_rle.argtypes = [u8p, i64, i64, ctypes.c_char_p, i64, i64]
        lib.dn_random_init.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.dn_random_next.argtypes = [ctypes.c_void_p]
        lib.dn_random_next.restype = ctypes.c_int32
        lib.dn_random_next_max.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.dn_random_next_max.restype = ctypes.c_int32
        u64p = ctypes.POINTER(ctypes.c_uint64)
        lib.fast_run.argtypes = [u64p, i64, i64, ctypes.c_int, i64, ctypes.c_int, i64, u64p,
                                 ctypes.POINTER(ctypes.c_int64)]
        lib.fast_hash.argtypes = [u64p, i64, i64]
        lib.fast_hash.restype = ctypes.c_uint64
        _C = lib
    return _C


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def c_run(b: np.ndarray, generations: int, boundary: int = TORUS) -> np.ndarray:
    lib = c_oracle()
    h, w = b.shape
    cur = np.ascontiguousarray(b, dtype=np.uint8).copy()
    scratch = np.empty_like(cur)
    rc = lib.oracle_run(_p(cur), _p(scratch), w, h, boundary, generations)
    if rc:
        raise ValueError("oracle_run rejected the board")
    return cur


def c_hash(b: np.ndarray) -> int:
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return int(c_oracle().oracle_hash(_p(b), b.shape[1], b.shape[0]))


def c_seed_dotnet(width: int, height: int, seed: int, mode: int = 0) -> np.ndarray:
    b = np.zeros((height, width), dtype=np.uint8)
    c_oracle().oracle_seed_dotnet(_p(b), width, height, seed, mode)
    return b


def c_seed_splitmix(width: int, height: int, seed: int) -> np.ndarray:
    b = np.zeros((height, width), dtype=np.uint8)
    c_oracle().oracle_seed_splitmix(_p(b), width, height, seed)
    return b


# ---------------------------------------------------------------- bit-packed long runs (gol_fast.c)
def pack64(b: np.ndarray) -> np.ndarray:
    """(H, W) uint8 cells -> (H, W/64) uint64, bit i of word j = cell 64j + i (W % 64 == 0)."""
    h, w = b.shape
    if w % 64:
        raise ValueError("pack64 needs W % 64 == 0")
    return np.packbits(np.ascontiguousarray(b, dtype=np.uint8), axis=1, bitorder="little").view("<u8").copy()


def unpack64(words: np.ndarray, width: int) -> np.ndarray:
    return np.unpackbits(words.view(np.uint8), axis=1, bitorder="little")[:, :width].astype(np.uint8)


def fast_run(b: np.ndarray, generations: int, boundary: int = TORUS, threads: int | None = None,
             every: int = 0):
    """gol_fast.c: run a W % 64 == 0 board `generations` steps on `threads` host threads.  Returns
    (final board (H, W) uint8, [(generation, hash, population)] every `every` generations)."""
    lib = c_oracle()
    h, w = b.shape
    words = pack64(b)
    n = generations // every if every > 0 else 0
    hashes = np.zeros(max(n, 1), np.uint64)
    pops = np.zeros(max(n, 1), np.int64)
    rc = lib.fast_run(words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), w, h, boundary, generations,
                      threads or (os.cpu_count() or 1), every,
                      hashes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                      pops.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
    if rc:
        raise ValueError("fast_run rejected the board")
    marks = [((i + 1) * every, int(hashes[i]), int(pops[i])) for i in range(n)]
    return unpack64(words, w), marks
