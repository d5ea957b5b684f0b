"""CPU restatement of the rows-on-lanes band pass (csrc/gol_lanes.hip), word for word, against the oracle.

The kernel's correctness rests on its data movement, which this restates in numpy on the same 32-bit words:
the plan (lanes_plan: window width, windows per band, bands), the window load (plain groups G0 + g, and G1 - g
bit-reversed for the mirrored half), the interleaved word order (word t bit b = cell M b + t), the DPP row moves
(wave_shr / wave_shl with zero fill, across the two halves' lane ranges), the seam between the halves (the
partner lane's cell 32 M - 1), the bounded masks, the LDS edge swap between windows (cells [32, 48) out, cells
[16, 32) in, bit 31 - j), the granule index of the hand-off, and the store.  The synchronous oracle
(GameOfLifeLogic.fs:59-63; torus GameOfLifeDriver.fs:21-25; bounded Script.fsx:6-13) is the reference; the GPU
tests (tests/test_gpu_lanes.py) check the kernel itself.
"""
import numpy as np
import pytest

import gol_oracle as O

MASK = 0xFFFFFFFF
WIN_ROWS, XCH_CELLS = 32, 16


def lanes_plan(W, H, k, m_opt=0):
    """gol_lanes.hip lanes_plan."""
    if W < 256 or W % 32 or W > 16384 or H < 3 or k < 1 or k > XCH_CELLS:
        return None
    if m_opt:
        m = m_opt if m_opt in (3, 5, 9, 17) else 0
    elif W <= 1024:
        m = 3 if W % 128 == 0 else 0
    else:
        m = 9 if W % 512 == 0 else (5 if W % 256 == 0 else 0)
    if not m:
        return None
    u = 64 * (m - 1)
    if W % u or W // u > 16:
        return None
    nx = W // u
    bmax = WIN_ROWS - 2 * k
    if bmax < k:
        return None
    nb = -(-H // bmax)
    most = H // k
    fill = -(-1024 // nx)
    if nb < fill:
        nb = min(fill, most)
    if nb > most or nb < 1 or -(-H // nb) > bmax:
        return None
    return m, nx, nb


def lut3(a, b, c, L):
    r = np.zeros_like(a)
    for idx in range(8):
        if (L >> idx) & 1:
            r |= (a if idx & 1 else ~a) & (b if idx & 2 else ~b) & (c if idx & 4 else ~c)
    return r


def life_next(sP, cP, sC, cC, sN, cN, alive):
    """gol_bitlogic.h life_next."""
    A = lut3(sP, sC, sN, 0x96)
    B = lut3(sP, sC, sN, 0xE8)
    X = lut3(cP, cC, cN, 0x96)
    Y = lut3(cP, cC, cN, 0xE8)
    o1 = lut3(A, Y, alive, 0x27)
    o2 = lut3(B, X, Y, 0x19)
    return lut3(o1, o2, A, 0x24)


def bitrev(v):
    v = v.astype(np.uint64)
    out = np.zeros_like(v)
    for i in range(32):
        out |= ((v >> np.uint64(i)) & np.uint64(1)) << np.uint64(31 - i)
    return out.astype(np.uint32)


def to_plain(board):
    H, W = board.shape
    bits = board.reshape(H, W // 32, 32).astype(np.uint64)
    return (bits << np.arange(32, dtype=np.uint64)).sum(axis=2).astype(np.uint32)


def from_plain(plain, W):
    H = plain.shape[0]
    bits = (plain[:, :, None].astype(np.uint64) >> np.arange(32, dtype=np.uint64)) & np.uint64(1)
    return bits.reshape(H, W).astype(np.uint8)


def lane_pass(board, gens, K, bounded, m_opt=0):
    H, W = board.shape
    m, nx, nb = lanes_plan(W, H, K, m_opt)
    M, U, nw = m, 64 * (m - 1), W // 32
    plain = to_plain(board)
    lane = np.arange(64)
    h, r = lane >> 5, lane & 31
    bands = []
    for band in range(nb):
        y0 = H * band // nb
        B = H * (band + 1) // nb - y0
        L = B + 2 * K
        wins = []
        for x in range(nx):
            G0, G1 = x * (U // 32) - 1, (x + 1) * (U // 32)
            p = np.zeros((64, M), np.uint32)
            for l in range(64):
                gy = y0 - K + r[l]
                for g in range(M):
                    G = G0 + g if h[l] == 0 else G1 - g
                    on = r[l] < L
                    if bounded and not (0 <= gy < H and 0 <= G < nw):
                        on = False
                    v = np.uint32(plain[gy % H, G % nw]) if on else np.uint32(0)
                    p[l, g] = bitrev(np.array([v]))[0] if h[l] else v
            w = np.zeros((64, M), np.uint32)
            for c in range(32 * M):
                w[:, c % M] |= ((p[:, c >> 5] >> np.uint32(c & 31)) & np.uint32(1)) << np.uint32(c // M)
            keepA = np.full(64, MASK, np.uint32)
            keepB = np.full(64, MASK, np.uint32)
            if bounded:
                q = 31 // M
                for l in range(64):
                    gy = y0 - K + r[l]
                    row_out = not 0 <= gy < H
                    col_out = (h[l] == 0 and x == 0) or (h[l] == 1 and x == nx - 1)
                    keepA[l] = 0 if row_out else (~((2 << q) - 1) & MASK if col_out else MASK)
                    keepB[l] = 0 if row_out else (~((1 << q) - 1) & MASK if col_out else MASK)
            wins.append({"w": w, "keepA": keepA, "keepB": keepB,
                         "edge": band == 0 or band == nb - 1 or x == 0 or x == nx - 1})
        bands.append({"y0": y0, "B": B, "L": L, "wins": wins})

    xch = {}

    def xrow(parity, b, side, e, x, hh):  # word t at + 2K t
        return ((((parity * nb + b) * 2 + side) * nx + x) * M) * (2 * K) + hh * K + e

    nblk = -(-gens // K)
    for blk in range(nblk):
        k = min(K, gens - blk * K)
        if blk > 0:
            par = (blk - 1) & 1
            for band, bd in enumerate(bands):
                up = band - 1 if band > 0 else (-1 if bounded else nb - 1)
                dn = band + 1 if band + 1 < nb else (-1 if bounded else 0)
                for x, win in enumerate(bd["wins"]):
                    for l in range(64):
                        src = None
                        if r[l] < K and up >= 0:
                            src = xrow(par, up, 1, r[l], x, h[l])
                        elif K + bd["B"] <= r[l] < bd["L"] and dn >= 0:
                            src = xrow(par, dn, 0, r[l] - K - bd["B"], x, h[l])
                        if src is not None:
                            win["w"][l] = [xch[(src + 2 * K * t, blk - 1)] for t in range(M)]
        for bd in bands:
            for win in bd["wins"]:
                w = win["w"]
                for _ in range(k):
                    above = np.vstack([np.zeros((1, M), np.uint32), w[:-1]])  # wave_shr:1, lane 0 <- 0
                    below = np.vstack([w[1:], np.zeros((1, M), np.uint32)])   # wave_shl:1, lane 63 <- 0
                    sv, cv = lut3(above, w, below, 0x96), lut3(above, w, below, 0xE8)
                    ps, pc = sv[lane ^ 32, M - 1], cv[lane ^ 32, M - 1]
                    sw0, cw0 = (sv[:, M - 1] << np.uint32(1)), (cv[:, M - 1] << np.uint32(1))
                    sel = (sv[:, 0] >> np.uint32(1)) | (ps & np.uint32(0x80000000))
                    cel = (cv[:, 0] >> np.uint32(1)) | (pc & np.uint32(0x80000000))
                    new = np.zeros_like(w)
                    for t in range(M):
                        new[:, t] = life_next(sv[:, t - 1] if t else sw0, cv[:, t - 1] if t else cw0, sv[:, t], cv[:, t],
                                              sv[:, t + 1] if t + 1 < M else sel, cv[:, t + 1] if t + 1 < M else cel,
                                              w[:, t])
                    if bounded and win["edge"]:
                        for t in range(M):
                            new[:, t] &= win["keepA"] if t <= 31 % M else win["keepB"]
                    w[:] = new
        if blk + 1 == nblk:
            break
        par = blk & 1
        for band, bd in enumerate(bands):
            slots = {}
            for x, win in enumerate(bd["wins"]):
                e = np.zeros(64, np.uint32)
                for i in range(XCH_CELLS):
                    c = 32 + i
                    e |= ((win["w"][:, c % M] >> np.uint32(c // M)) & np.uint32(1)) << np.uint32(i)
                slots[x] = e
            for x, win in enumerate(bd["wins"]):
                w = win["w"]
                for l in range(64):
                    xn = x - 1 if h[l] == 0 else x + 1
                    on = True
                    if not 0 <= xn < nx:
                        on = not bounded
                        xn %= nx
                    v = int(slots[xn][l ^ 32]) if on else 0  # the neighbour's other half, same row
                    for j in range(32 - XCH_CELLS, 32):
                        t, b, s = j % M, j // M, 31 - j
                        bit = (v >> s) & 1
                        w[l, t] = (int(w[l, t]) & ~(1 << b) & MASK) | (bit << b)
            for x, win in enumerate(bd["wins"]):
                for l in range(64):
                    for side in range(2):
                        e = r[l] - K if side == 0 else r[l] - bd["B"]
                        if 0 <= e < K and r[l] < bd["L"]:
                            base = xrow(par, band, side, e, x, h[l])
                            for t in range(M):
                                assert (base + 2 * K * t, blk) not in xch  # every granule written once per block
                                xch[(base + 2 * K * t, blk)] = win["w"][l, t]
    out = np.zeros((H, nw), np.uint32)
    for bd in bands:
        for x, win in enumerate(bd["wins"]):
            G0, G1 = x * (U // 32) - 1, (x + 1) * (U // 32)
            w = win["w"]
            for l in range(64):
                if not K <= r[l] < K + bd["B"]:
                    continue
                for g in range(1, M):
                    p = 0
                    for i in range(32):
                        c = 32 * g + i
                        p |= ((int(w[l, c % M]) >> (c // M)) & 1) << i
                    G = G0 + g if h[l] == 0 else G1 - g
                    out[bd["y0"] + r[l] - K, G] = bitrev(np.array([p], np.uint32))[0] if h[l] else p
    return from_plain(out, W)


def test_plan_of_config2():
    assert lanes_plan(4096, 4096, 8) == (9, 8, 256)
    assert lanes_plan(4096, 4096, 12) is None  # 32 - 2k < k
    assert lanes_plan(4096, 4096, 8, 17) == (17, 4, 256)


@pytest.mark.parametrize("bounded", [False, True])
@pytest.mark.parametrize("W,H,K,m,gens", [(512, 40, 8, 0, 19), (1024, 48, 4, 0, 13), (768, 30, 3, 0, 11),
                                          (256, 24, 5, 5, 12), (1024, 36, 8, 17, 17), (384, 30, 8, 3, 18)])
def test_lane_pass_restatement_matches_oracle(W, H, K, m, gens, bounded):
    board = (np.random.default_rng(W + H + K + bounded).random((H, W)) < 0.4).astype(np.uint8)
    got = lane_pass(board, gens, K, bounded, m)
    want = O.c_run(board, gens, 1 if bounded else 0)
    np.testing.assert_array_equal(got, want)
