"""GPU parity of the LDS-resident small-board pass (csrc/gol_resident.hip).

Boards up to 2^17 cells (packed ilv 1; with the cooperative pass off, board option "coop" 0) or 2^14 cells (byte layout,
widths not a multiple of 32) run a whole gol_step call as one launch with the board held in one workgroup's LDS; the kernel itself takes
up to 2^19 / 2^16 cells, which these tests reach with the "resident_max_cells" option raised.  Bar: bit-exact against the oracle
(GameOfLifeLogic.fs:56-63 rule, torus GameOfLifeDriver.fs:21-25, bounded Script.fsx:6-13) and against the
streaming pass on the same board ("resident_max_cells" 0 forces the streaming pass).  The single-wave pass
("wave_resident") is off in these runs so the shapes it would take exercise the pass they name.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _rand(h, w, seed, p=0.5):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


def _run(gol, b0, boundary, steps, resident):
    # the single-wave and cooperative passes (taken first by default) are off here: LDS-resident vs streaming
    # (resident_max_cells 0 forces the streaming pass, or the byte step on a ragged board)
    h, w = b0.shape
    opts = {"resident_max_cells": (1 << 20) if resident else 0, "coop": 0, "wave_resident": 0}
    with gol.Board(w, h, boundary, options=opts) as b:
        b.set_cells(b0)
        for g in steps:
            b.step(g)
        assert b.generation == sum(steps)
        return b.get_cells()


# (w, h): packed boards (w % 32 == 0) from one word per row to the 2^19-cell capacity, byte boards
# (ragged widths) from the 3x3 minimum (gol_create) to the 2^16-cell capacity
SHAPES = [(32, 3), (32, 7), (64, 3), (96, 40), (256, 256), (1024, 512), (512, 1024),
          (3, 3), (5, 4), (3, 11), (100, 100), (33, 17), (255, 257)]


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", SHAPES)
def test_resident_matches_oracle_and_streaming(gol, oracle, w, h, boundary):
    b0 = _rand(h, w, 7 * w + h + boundary)
    steps = [1, 37, 0, 62]  # several calls: the resident launch ping-pongs the board buffers
    want = oracle.run(b0, sum(steps), boundary)
    got = _run(gol, b0, boundary, steps, resident=True)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(_run(gol, b0, boundary, steps, resident=False), want)


@pytest.mark.parametrize("boundary", [0, 1])
def test_resident_long_run(gol, oracle, boundary):
    # 256^2 bounded / torus over 3000 generations in one call (BASELINE config-5 style long run)
    b0 = _rand(256, 256, 5150 + boundary, p=0.3)
    np.testing.assert_array_equal(_run(gol, b0, boundary, [3000], resident=True), oracle.run(b0, 3000, boundary))


def test_resident_byte_input_values_normalised(gol, oracle):
    # nonzero = alive on input (set_cells bytes), 0/1 after a step, as on the per-generation byte kernel
    w, h = 50, 40
    b0 = _rand(h, w, 99) * np.uint8(255)
    got = _run(gol, b0, 0, [5], resident=True)
    np.testing.assert_array_equal(got, oracle.run((b0 != 0).astype(np.uint8), 5, 0))


# ---------------------------------------------------------------- single-wave register-resident pass
def _run_wave(gol, b0, boundary, steps, wave):
    h, w = b0.shape
    with gol.Board(w, h, boundary, options={"wave_resident": int(wave)}) as b:
        b.set_cells(b0)
        for g in steps:
            b.step(g)
        assert b.generation == sum(steps)
        return b.get_cells()


# ragged (byte boards) and packed widths up to 128, heights up to 256 with 1-4 rows per lane; the
# reference's own 100 x 100 board first (GameOfLifeLogic.fs:5)
WAVE_SHAPES = [(100, 100), (3, 3), (5, 4), (33, 17), (97, 99), (127, 64), (128, 128), (64, 200), (32, 256),
               (100, 3), (31, 192), (65, 130)]


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", WAVE_SHAPES)
def test_wave_resident_matches_oracle_and_other_paths(gol, oracle, w, h, boundary):
    b0 = _rand(h, w, 11 * w + h + boundary, p=0.4)
    steps = [1, 40, 0, 59]
    want = oracle.run(b0, sum(steps), boundary)
    np.testing.assert_array_equal(_run_wave(gol, b0, boundary, steps, wave=True), want)
    np.testing.assert_array_equal(_run_wave(gol, b0, boundary, steps, wave=False), want)


@pytest.mark.parametrize("boundary", [0, 1])
def test_wave_resident_long_run_reference_board(gol, oracle, boundary):
    """The reference's board, .NET Random seed 42 in its order (GameOfLifeDriver.fs:9-19), 5000 generations
    in one call, against the C oracle."""
    b0 = oracle.seed_dotnet(100, 100, 42, 0)
    np.testing.assert_array_equal(_run_wave(gol, b0, boundary, [5000], wave=True), oracle.c_run(b0, 5000, boundary))


def test_wave_resident_byte_values_normalised(gol, oracle):
    b0 = _rand(100, 100, 3) * np.uint8(77)
    np.testing.assert_array_equal(_run_wave(gol, b0, 0, [3], wave=True), oracle.run((b0 != 0).astype(np.uint8), 3, 0))
