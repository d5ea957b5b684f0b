"""CPU check of the cooperative pass's block schedule (csrc/gol_coop.hip), against the oracle.

The kernel's correctness rests on its schedule: balanced bands of >= K rows, K halo rows per side, generation j
of a block of k producing local rows [K - k + 1 + j, K + B + k - 1 - j), and the hand-off of each band's first
and last K rows through a parity-double-buffered exchange (a band shorter than 2K rows sends some rows to both
sides).  This restates that schedule on byte boards, band by band, and checks it against the synchronous
oracle (GameOfLifeLogic.fs:59-63; torus GameOfLifeDriver.fs:21-25; bounded Script.fsx:6-13).  The GPU tests
(tests/test_gpu_coop.py) check the kernel itself.
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
