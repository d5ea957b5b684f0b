"""GPU parity of the seam geometry of the streaming pass (csrc/gol_step.hip, DESIGN.md 4.1 "Seam strips").

On a torus the deep passes cover a row with strips of 63 stored blocks whose 64th lane (the seam lane) holds both
halos -- half of the block right of the strip and half of the block left of it -- and the blocks left over
(nblocks mod 63) in remainder waves that pack several row segments' sub-strips side by side, each at its own row
offset.  Bar: bit-exact against the oracle (GameOfLifeLogic.fs:59-63 rule, torus GameOfLifeDriver.fs:21-25) and
against the halo-lane geometry (board option "seam" -1) on the same board, for every layout, strip-count
boundaries (nblocks around multiples of 63), remainders of every packing (1 to 21 sub-strips per wave), many
short segments (board option "seg_rows": packed remainder units, the short last segment), SIMD-group splits and
the ghost-row strips of the multi-GPU path.
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


def _run(gol, b0, k, ilv, opts):
    h, w = b0.shape
    with gol.Board(w, h, gol.TORUS, tblock_k=k, ilv=ilv, options=dict(opts, coop=0)) as b:
        assert b.info()["tblock_k"] == k
        b.set_cells(b0).step(2 * k + 5)
        return b.get_cells()


@pytest.mark.parametrize("ilv,k", [(1, 8), (1, 16), (2, 12), (2, 16), (2, 8), (4, 8), (4, 6)])
@pytest.mark.parametrize("nblocks", [63, 64, 65, 94, 125, 126, 127, 189, 200])
def test_seam_strips_match_oracle(gol, oracle, ilv, k, nblocks):
    w = 32 * ilv * nblocks
    h = 203  # segments of 24 rows: 9 segments, the last one short (11 rows) -- shorter than k for k >= 12
    b0 = _rand(h, w, nblocks * 31 + ilv * 7 + k)
    want = oracle.c_run(b0, 2 * k + 5, 0)
    for opts in ({}, {"seg_rows": 24}, {"seg_rows": 24, "split": -1}, {"seam": -1, "seg_rows": 24}):
        np.testing.assert_array_equal(_run(gol, b0, k, ilv, opts), want, err_msg=str(opts))


@pytest.mark.parametrize("seg_rows", [16, 40])
@pytest.mark.parametrize("h", [97, 160, 333])
def test_seam_remainder_packing_segments(gol, oracle, seg_rows, h):
    """rem = 16 blocks (a 65536-wide row's geometry at 1/16 the width: 1024 + 16 blocks), three sub-strips per
    remainder wave, every way the segments fall into packed and lone remainder units."""
    w = 64 * (63 * 2 + 16)
    b0 = _rand(h, w, h + seg_rows)
    for k in (12, 16):
        want = oracle.c_run(b0, 2 * k + 5, 0)
        np.testing.assert_array_equal(_run(gol, b0, k, 2, {"seg_rows": seg_rows}), want, err_msg=f"k={k}")


def test_seam_ghost_row_strips(gol, oracle):
    """The multi-GPU rank kernel (ghost-row strips, gol_strip_step) with seam strips and packed remainders: 3 strips
    in one process against the oracle."""
    import torch

    from gameoflifewithactors_amd.strips import LocalBoard

    w, h, k = 64 * 140, 600, 12
    b0 = _rand(h, w, 5)
    lb = LocalBoard(w, h, 0, k, 3)
    lb.set_cells(torch.as_tensor(b0))
    lb.step(3 * k + 1)
    np.testing.assert_array_equal(lb.get_cells().numpy(), oracle.c_run(b0, 3 * k + 1, 0))


@pytest.mark.parametrize("seg_rows", [4, 8, 11])
def test_seam_segments_shorter_than_k(gol, oracle, seg_rows):
    """segments shorter than k (the "seg_rows" option accepts any length) must not be packed into
    remainder waves -- sub-strip j reads its rows at a fixed offset from sub-strip 0's walk, so segment 1's first
    rows would wrap.  Such segments run as lone remainder units; the board is still exact, on the single board and on
    the ghost-row strips of a multi-part board (whose strip launches take the board's options too)."""
    w, h, k = 64 * (63 * 2 + 16), 150, 12
    b0 = _rand(h, w, 300 + seg_rows)
    want = oracle.c_run(b0, 2 * k + 5, 0)
    np.testing.assert_array_equal(_run(gol, b0, k, 2, {"seg_rows": seg_rows}), want)
    with gol.Board(w, h, gol.TORUS, tblock_k=k, ilv=2, devices=[0, 0], options={"seg_rows": seg_rows}) as b:
        assert b.get_option("seg_rows") == seg_rows
        b.set_cells(b0).step(2 * k + 5)
        np.testing.assert_array_equal(b.get_cells(), want)
