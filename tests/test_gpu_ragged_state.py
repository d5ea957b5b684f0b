"""GPU parity of a ragged byte board whose state stays in whole-word scratch rows between gol_step calls
(csrc/gol_capi.cpp rag_state; DESIGN.md 4.1 "Ragged rows").

The streaming and cooperative passes on ragged boards (width not a multiple of 32: the reference's `size` is any
integer, GameOfLifeLogic.fs:5) pack the byte board into scratch words once and leave the state there after the call;
every other access -- readbacks (cells, Gray8, region, hash, population, snapshot), RLE placement, a call that takes
another pass (short calls, a changed option) -- first brings the bytes up to date, and overwrites (set_cells, seed,
clear, load) drop the scratch state.  Bar: bit-exact against the oracle (rule GameOfLifeLogic.fs:59-63, torus
GameOfLifeDriver.fs:21-25, bounded Script.fsx:6-13) after every kind of interleaving.
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


# (w, h): the streaming pass (wider than 8192) and the cooperative pass (<= 8192 wide, <= 2^26 cells)
BOARDS = [(8209, 40), (1001, 300)]


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", BOARDS)
def test_readbacks_between_calls(gol, oracle, w, h, boundary):
    b0 = _rand(h, w, w + h + boundary)
    with gol.Board(w, h, boundary) as b:
        b.set_cells(b0)
        gen, cur = 0, b0
        for g in (20, 16, 3, 40, 1, 17):  # multi-generation passes, a short byte-step call, a single generation
            b.step(g)
            gen += g
            cur = oracle.c_run(cur, g, boundary)
            np.testing.assert_array_equal(b.get_cells(), cur, err_msg=f"gen {gen}")
            assert b.population() == int(cur.sum())
            np.testing.assert_array_equal(b.get_region(5, 3, 33, 7), cur[3:10, 5:38])
        assert b.generation == gen


@pytest.mark.parametrize("w,h", BOARDS)
def test_hash_render_snapshot_rle_between_calls(gol, oracle, w, h):
    b0 = _rand(h, w, 7 * w + h)
    with gol.Board(w, h, 0) as b, gol.Board(w, h, 0, options={"ragged_stream": 0, "coop": 0}) as ref:
        b.set_cells(b0)
        ref.set_cells(b0)
        b.step(24)
        ref.step(24)
        assert b.hash() == ref.hash()  # the first access after the pass: a reduction
        b.step(24)
        ref.step(24)
        np.testing.assert_array_equal(b.render_gray8(255, stride=w + 3), ref.render_gray8(255, stride=w + 3))
        b.step(24)
        ref.step(24)
        np.testing.assert_array_equal(b.save_packed(), ref.save_packed())
        b.step(24)
        ref.step(24)
        b.place_rle("bo$2bo$3o!", 11, 5)  # a glider onto the scratch-held state
        ref.place_rle("bo$2bo$3o!", 11, 5)
        b.step(30)
        ref.step(30)
        np.testing.assert_array_equal(b.get_cells(), ref.get_cells())
        want = oracle.c_run(b0, 96, 0)
        glider = np.zeros_like(want)
        for (dx, dy) in ((1, 0), (2, 1), (0, 2), (1, 2), (2, 2)):
            glider[5 + dy, 11 + dx] = 1
        want = oracle.c_run(np.maximum(want, glider), 30, 0)
        np.testing.assert_array_equal(ref.get_cells(), want)


@pytest.mark.parametrize("w,h", BOARDS)
def test_overwrites_and_option_changes_between_calls(gol, oracle, w, h):
    b0 = _rand(h, w, 3 * w + h)
    b1 = _rand(h, w, 5 * w + h)
    with gol.Board(w, h, 1) as b:
        b.set_cells(b0).step(20)
        b.set_cells(b1)  # overwrite while the scratch rows hold the state: they must not come back
        b.step(20)
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b1, 20, 1))
        b.step(12)
        b.clear()
        b.step(8)
        assert b.population() == 0
        b.set_cells(b0).step(16)
        b.set_option("ragged_stream", 0).set_option("coop", 0)  # next call: the byte step on the bytes
        b.step(8)
        b.set_option("ragged_stream", 1).set_option("coop", 1)
        b.step(16)
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 40, 1))
        b.step(20)
        b.seed_splitmix(99)  # overwrite by seeding
        with gol.Board(w, h, 1) as fresh:
            fresh.seed_splitmix(99)
            assert b.hash() == fresh.hash()
