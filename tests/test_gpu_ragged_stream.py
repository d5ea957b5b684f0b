"""GPU parity of ragged boards on the streaming pass (torus: ring rows on the aligned kernel, gol_formats.hip
gol_pack_ring / gol_ring_refresh; bounded: column-masked block rows) from 3 * 2^26 cells (board option "ragged_ring"
1, the default; 2 forces them on any size, as these tests do), below that the M = 1 kRagged variant of
csrc/gol_step.hip ("ragged_ring" 0 everywhere; DESIGN.md 4.1 "Ragged rows").

The reference's board size is any integer (GameOfLifeLogic.fs:5, GameofLife.fs:18).  Byte boards whose width is not
a multiple of 32 and that the cooperative pass does not take (wider than 8192 cells or above 2^26 cells) run the
streaming pass on whole-word scratch rows: the row end closed at bit level on a torus (the west neighbour of cell 0
is cell W - 1: GameOfLifeDriver.fs:21-25), dead beyond the last cell when bounded (Script.fsx:6-13).  Bar:
bit-exact against the oracle and against the per-generation byte step (board option "ragged_stream" 0), for
last words of 1 to 31 cells, strip-count boundaries (words around multiples of 62), every depth and split calls.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _rand(h, w, seed, p=0.4):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


def _run(gol, b0, boundary, steps, stream, tblock_k=0, ring=1):
    h, w = b0.shape
    with gol.Board(w, h, boundary, tblock_k=tblock_k, options={"ragged_stream": int(stream), "ragged_ring": ring}) as b:
        assert not b.info()["packed"]
        b.set_cells(b0)
        for g in steps:
            b.step(g)
        assert b.generation == sum(steps)
        return b.get_cells()


# widths past the cooperative pass (> 8192): last words of 1, 17, 31 cells; words around 62 * n (the strip count
# boundaries of the ring geometry, 62 * 133 + 1 = 8247 words: one more strip so the partial word is never a halo)
WIDTHS = [8193, 8209, 8223, 10001, 62 * 133 * 32 - 31, 62 * 134 * 32 + 5, 16383]


@pytest.mark.parametrize("boundary,ring", [(0, 2), (0, 0), (1, 2), (1, 0), (0, 1)])
@pytest.mark.parametrize("w", WIDTHS)
def test_ragged_stream_matches_oracle(gol, oracle, w, boundary, ring):
    h = 70
    b0 = _rand(h, w, w + boundary)
    steps = [21, 3, 16]  # 16 + 4 + 1, the byte step for the 3-generation call, 16
    want = oracle.c_run(b0, sum(steps), boundary)
    np.testing.assert_array_equal(_run(gol, b0, boundary, steps, stream=True, ring=ring), want)


# ring rows at ilv 2 (above 2^25 ring cells): the widths' last 64-cell block holds 1 .. 63 of the board's cells, the
# seam geometry (>= 63 blocks) and not
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w", [8193, 8255, 10001, 16383, 16447, 4033 * 8 + 1])
def test_ragged_ring_interleaved(gol, oracle, w, boundary):
    """Block rows at ilv 2 against the ilv-1 rows and the oracle's light cone.  Bounded: edge-fill strips whose last
    block is partial (1 .. 63 of its cells on the board), masked at every level (gol_step.hip NARROW = 2)."""
    h = (1 << 25) // w + 40
    b0 = _rand(h, w, w, p=0.3)
    with gol.Board(w, h, boundary, options={"coop": 0, "ragged_ring": 2}) as b:  # below the size rule: forced
        assert b.info()["tblock_k"] == 16
        b.set_cells(b0).step(16 + 12 + 5)
        got_rows = b.get_region(0, 0, w, 64)
        got_end = b.get_region(0, h - 40, w, 40)
        b.set_option("ragged_ring", 0)
        b.set_cells(b0).step(16 + 12 + 5)
        np.testing.assert_array_equal(b.get_region(0, 0, w, 64), got_rows)
        np.testing.assert_array_equal(b.get_region(0, h - 40, w, 40), got_end)
    gens = 33
    if boundary == 0:
        # the first 64 rows against the oracle's light cone (the torus rows wrap: rows h-33 .. h-1 above row 0)
        win = np.concatenate([b0[h - gens:], b0[:64 + gens]], axis=0)
        sub = oracle.c_run(np.ascontiguousarray(win), gens, 0)  # the window's own y wrap only pollutes the cone edges
        np.testing.assert_array_equal(got_rows, sub[gens:gens + 64])
    else:
        # bounded: rows 0..63 depend only on rows 0..63+gens (dead above the board); bounded x edges are exact
        sub = oracle.c_run(np.ascontiguousarray(b0[:64 + gens]), gens, 1)
        np.testing.assert_array_equal(got_rows, sub[:64])


@pytest.mark.parametrize("k", [1, 2, 8, 16, 24, 32])
def test_ragged_stream_depths(gol, oracle, k):
    w, h = 9001, 64
    b0 = _rand(h, w, k)
    for boundary in (0, 1):
        want = oracle.c_run(b0, 2 * k + 5, boundary)
        np.testing.assert_array_equal(_run(gol, b0, boundary, [2 * k + 5], stream=True, tblock_k=k), want,
                                      err_msg=f"boundary={boundary}")


def test_ragged_stream_equals_byte_step(gol):
    """The two paths of a ragged board agree on a larger board (no oracle: both are checked against it above)."""
    w, h = 12001, 900
    b0 = _rand(h, w, 3)
    for boundary in (0, 1):
        a = _run(gol, b0, boundary, [37], stream=True)
        b = _run(gol, b0, boundary, [37], stream=False)
        np.testing.assert_array_equal(a, b)


def test_ragged_stream_large_board(gol, oracle):
    """10001 x 10001 torus (above 2^26 cells): a light-cone window of the oracle (exact: no cell within `gens` of
    the window's interior depends on anything outside it) plus the torus wrap at the row end (columns 0 and W-1)."""
    w = h = 10001
    gens = 40
    b0 = _rand(h, w, 77, p=0.3)
    got = _run(gol, b0, 0, [gens], stream=True)
    # window around the row end: columns W-100 .. W-1 and 0 .. 99, rows 5000 .. 5199 (a torus: rolling is exact)
    win = np.roll(b0, 100, axis=1)[5000 - gens:5200 + gens, :200 + gens]
    sub = oracle.c_run(np.ascontiguousarray(np.pad(win, 0)), gens, 1)
    np.testing.assert_array_equal(np.roll(got, 100, axis=1)[5000:5200, gens:200], sub[gens:200 + gens, gens:200])


@pytest.mark.parametrize("calls", [[100], [32, 32, 32, 4, 32]])
def test_ring_refresh_long_ring_state(gol, oracle, calls):
    """torus ring rows kept in one ring state past 64 generations, so the refresh of the copies at both
    ends of every row (gol_ring_refresh, whenever ring_age + k would pass the 64 copied cells) runs between passes --
    one 100-generation call, and 32-generation calls whose state stays in the ring rows between them (the 4-generation
    call is the streaming pass too: >= 4 generations).  Against the oracle and the ilv-1 rows ("ragged_ring" 0)."""
    w, h = 8209, 70
    b0 = _rand(h, w, 808)
    want = oracle.c_run(b0, sum(calls), 0)
    np.testing.assert_array_equal(_run(gol, b0, 0, calls, stream=True, ring=2), want)
    np.testing.assert_array_equal(_run(gol, b0, 0, calls, stream=True, ring=0), want)
