# CPU emulation of gol_coop.hip's block schedule (bands, K-row halos, parity exchange, shrinking valid rows),
# checked against the oracle on small boards: the logic check that preceded the GPU parity tests.
# Emulates gol_band_pass's schedule (bands, waves' row slices, trapezoid, parity exchange) on byte boards.
import numpy as np, sys
sys.path.insert(0, '/root/repo/oracle')
import gol_oracle as O

def life_rows(P, C, N, bounded):
    # next state of row C given rows P, C, N (1-D arrays), horizontal torus/bounded
    def hs(r):
        if bounded:
            l = np.concatenate([[0], r[:-1]]); rr = np.concatenate([r[1:], [0]])
        else:
            l = np.roll(r, 1); rr = np.roll(r, -1)
        return l + r + rr
    t = hs(P) + hs(C) + hs(N)
    return ((t == 3) | ((t == 4) & (C == 1))).astype(np.uint8)

def band_pass(board, gens, K, nwg, bounded, R=None, W16=16):
    H, Wd = board.shape
    out = np.zeros_like(board)
    xch = {}
    flags = [0]*nwg
    # run bands in lockstep per block (the protocol's ordering guarantees equivalence)
    bands = []
    for b in range(nwg):
        y0 = H*b//nwg; y1 = H*(b+1)//nwg; B = y1-y0; L = B+2*K
        rows = np.zeros((L, Wd), np.uint8)
        for i in range(L):
            gy = y0-K+i
            if bounded and not (0 <= gy < H): continue
            rows[i] = board[gy % H]
        bands.append([y0, B, L, rows])
    nblk = (gens+K-1)//K
    for blk in range(nblk):
        k = min(K, gens-blk*K)
        if blk > 0:
            par = (blk-1) & 1
            for b,(y0,B,L,rows) in enumerate(bands):
                up = b-1 if b > 0 else (-1 if bounded else nwg-1)
                dn = b+1 if b+1 < nwg else (-1 if bounded else 0)
                for li in range(L):
                    if li < K and up >= 0: rows[li] = xch[(par, up, 1, li)]
                    elif li >= K+B and dn >= 0: rows[li] = xch[(par, dn, 0, li-K-B)]
        for b,(y0,B,L,rows) in enumerate(bands):
            for j in range(k):
                lo, hi = K-k+1+j, K+B+k-1-j
                new = rows.copy()
                for i in range(lo, hi):
                    gy = y0-K+i
                    if bounded and not (0 <= gy < H): new[i] = 0; continue
                    new[i] = life_rows(rows[i-1], rows[i], rows[i+1], bounded)
                rows[:] = new
        if blk+1 == nblk: break
        par = blk & 1
        for b,(y0,B,L,rows) in enumerate(bands):
            for li in range(L):
                for side in range(2):
                    e = li-K if side == 0 else li-B
                    if 0 <= e < K: xch[(par, b, side, e)] = rows[li].copy()
    for (y0,B,L,rows) in bands:
        out[y0:y0+B] = rows[K:K+B]
    return out

rng = np.random.default_rng(1)
for (H, Wd, K, bounded, gens) in [(64, 40, 8, False, 37), (64, 40, 8, True, 37), (50, 33, 3, False, 20), (48, 32, 16, False, 40), (20, 32, 8, False, 17), (300, 64, 16, True, 33), (16, 32, 8, False, 24)]:
    nwg = min(256, H//K)
    b0 = (rng.random((H, Wd)) < 0.4).astype(np.uint8)
    want = b0.copy()
    for g in range(gens):
        want = O.step(want, 1 if bounded else 0)
    got = band_pass(b0, gens, K, nwg, bounded)
    print(H, Wd, K, bounded, gens, nwg, 'OK' if np.array_equal(got, want) else 'MISMATCH %d' % (got != want).sum())
