"""CPU check of the cooperative pass's block schedule (csrc/gol_coop.hip), against the oracle.

The kernel's correctness rests on its schedule: balanced bands of >= K rows, K halo rows per side, generation j
of a block of k producing local rows [K - k + 1 + j, K + B + k - 1 - j), and the hand-off of each band's first
and last K rows through a parity-double-buffered exchange (a band shorter than 2K rows sends some rows to both
sides).  This restates that schedule on byte boards, band by band, and checks it against the synchronous
oracle (GameOfLifeLogic.fs:59-63; torus GameOfLifeDriver.fs:21-25; bounded Script.fsx:6-13).  The GPU tests
(tests/test_gpu_coop.py) check the kernel itself.  The ragged word layout of the pass (widths not a multiple of 32,
rows padded to whole words, the row end patched at bit level) is restated word by word at the end.
"""
import numpy as np
import pytest

import gol_oracle as O


def _next_row(P, C, N, bounded):
    def hs(r):
        if bounded:
            return np.concatenate([[0], r[:-1]]) + r + np.concatenate([r[1:], [0]])
        return np.roll(r, 1) + r + np.roll(r, -1)

    t = hs(P) + hs(C) + hs(N)
    return ((t == 3) | ((t == 4) & (C == 1))).astype(np.uint8)


def band_schedule(board, gens, K, nwg, bounded):
    H, W = board.shape
    xch = {}
    bands = []
    for b in range(nwg):
        y0, y1 = H * b // nwg, H * (b + 1) // nwg
        B = y1 - y0
        rows = np.zeros((B + 2 * K, W), np.uint8)
        for i in range(B + 2 * K):
            gy = y0 - K + i
            if not bounded or 0 <= gy < H:
                rows[i] = board[gy % H]
        bands.append((y0, B, rows))
    nblk = (gens + K - 1) // K
    for blk in range(nblk):
        k = min(K, gens - blk * K)
        if blk > 0:  # halo rows from the neighbours' exchange rows of the previous block
            par = (blk - 1) & 1
            for b, (y0, B, rows) in enumerate(bands):
                up = b - 1 if b > 0 else (-1 if bounded else nwg - 1)
                dn = b + 1 if b + 1 < nwg else (-1 if bounded else 0)
                for i in range(K):
                    if up >= 0:
                        rows[i] = xch[(par, up, 1, i)]
                    if dn >= 0:
                        rows[K + B + i] = xch[(par, dn, 0, i)]
        for y0, B, rows in bands:
            for j in range(k):
                new = rows.copy()
                for i in range(K - k + 1 + j, K + B + k - 1 - j):
                    gy = y0 - K + i
                    dead = bounded and not 0 <= gy < H
                    new[i] = 0 if dead else _next_row(rows[i - 1], rows[i], rows[i + 1], bounded)
                rows[:] = new
        if blk + 1 < nblk:  # hand-off: first and last K rows of every band
            for b, (y0, B, rows) in enumerate(bands):
                for i in range(K):
                    xch[(blk & 1, b, 0, i)] = rows[K + i].copy()
                    xch[(blk & 1, b, 1, i)] = rows[B + i].copy()
    out = np.zeros_like(board)
    for y0, B, rows in bands:
        out[y0:y0 + B] = rows[K:K + B]
    return out


@pytest.mark.parametrize("H,W,K,gens", [(64, 40, 8, 37), (50, 33, 3, 20), (48, 32, 16, 40), (20, 32, 8, 17),
                                        (16, 32, 8, 24), (90, 64, 16, 33)])
@pytest.mark.parametrize("bounded", [False, True])
def test_band_schedule_matches_oracle(H, W, K, gens, bounded):
    b0 = (np.random.default_rng(H * W + K).random((H, W)) < 0.4).astype(np.uint8)
    want = O.run(b0, gens, 1 if bounded else 0)
    got = band_schedule(b0, gens, K, min(256, H // K), bounded)
    np.testing.assert_array_equal(got, want)


# ---------------------------------------------------------------- ragged rows (kLayRagged)
M32 = 0xFFFFFFFF


def _ragged_row_sums(words, W, M, bounded):
    """Per word of a ragged row (nwp = len(words) words, lane l holding words [l M, l M + M)): the horizontal
    3-sums {s, c} as gol_coop.hip's ragged_row_sum computes them: west / east words from the word itself and its
    neighbours (zero beyond the row's words, as the zero-fill lane moves give), then on a torus the two row-end
    words patched: the west neighbour of cell 0 is bit lb of the last word, the east neighbour of cell W - 1 is
    bit 0 of word 0 (GameOfLifeDriver.fs:21-25)."""
    nwp = len(words)
    last = (W + 31) // 32 - 1
    lb = (W - 1) & 31
    s = np.zeros(nwp, np.uint64)
    c = np.zeros(nwp, np.uint64)
    for g in range(nwp):
        w = int(words[g])
        left = int(words[g - 1]) if g > 0 else 0
        right = int(words[g + 1]) if g + 1 < nwp else 0
        west = ((w << 1) | (left >> 31)) & M32
        east = ((w >> 1) | (right << 31)) & M32
        if not bounded:
            if g == 0:
                west = ((w << 1) | ((int(words[last]) >> lb) & 1)) & M32
            if g == last:
                east = (w >> 1) | ((int(words[0]) & 1) << lb)
        s[g] = west ^ w ^ east
        c[g] = (west & w) | (west & east) | (w & east)
    return s, c


def ragged_step(rows_words, W, M, bounded):
    """One generation of a ragged board held as whole words (rows_words: H x nwp uint32), the cooperative pass's
    kLayRagged layout: row sums per word, the rule per cell from three rows' sums, every word masked to the row's
    cells (wmask)."""
    H, nwp = rows_words.shape
    assert nwp % M == 0 and nwp // M <= 64
    last = (W + 31) // 32 - 1
    lb = (W - 1) & 31
    lastmask = M32 if lb == 31 else (2 << lb) - 1
    wmask = [M32 if g < last else (lastmask if g == last else 0) for g in range(nwp)]
    sums = [_ragged_row_sums(rows_words[y], W, M, bounded) for y in range(H)]
    bits = np.arange(32, dtype=np.uint64)

    def cellsum(y):
        if bounded and not 0 <= y < H:
            return np.zeros((nwp, 32), np.int64)
        s, c = sums[y % H]
        return ((s[:, None] >> bits) & 1).astype(np.int64) + 2 * ((c[:, None] >> bits) & 1).astype(np.int64)

    out = np.zeros_like(rows_words)
    for y in range(H):
        t = cellsum(y - 1) + cellsum(y) + cellsum(y + 1)
        ctr = ((rows_words[y].astype(np.uint64)[:, None] >> bits) & 1).astype(np.int64)
        alive = (t == 3) | ((t == 4) & (ctr == 1))
        packed = (alive.astype(np.uint64) << bits).sum(axis=1)
        out[y] = (packed & np.array(wmask, np.uint64)).astype(np.uint32)
    return out


@pytest.mark.parametrize("W,M", [(33, 1), (100, 1), (2047, 1), (2049, 2), (4095, 2), (4097, 4), (8191, 4)])
@pytest.mark.parametrize("bounded", [False, True])
def test_ragged_row_layout_matches_oracle(W, M, bounded):
    """The ragged word layout and its row-end fix-up (words padded to a multiple of M, cells past W kept dead),
    restated word by word, against the oracle over a few generations."""
    H = 6
    nw = (W + 31) // 32
    nwp = (nw + M - 1) // M * M
    b0 = (np.random.default_rng(W + M).random((H, W)) < 0.4).astype(np.uint8)
    rows = np.zeros((H, nwp), np.uint32)
    for y in range(H):
        for x in np.nonzero(b0[y])[0]:
            rows[y, x // 32] |= np.uint32(1 << (x % 32))
    cur = rows
    gens = 3
    for _ in range(gens):
        cur = ragged_step(cur, W, M, bounded)
    got = np.zeros((H, W), np.uint8)
    for y in range(H):
        for x in range(W):
            got[y, x] = (int(cur[y, x // 32]) >> (x % 32)) & 1
    np.testing.assert_array_equal(got, O.run(b0, gens, 1 if bounded else 0))
