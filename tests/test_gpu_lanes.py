"""GPU parity of the rows-on-lanes band pass (csrc/gol_lanes.hip, board option "lanes").

A wave owns a window of a band -- all its rows on the lanes, 64 (m - 1) useful columns plus 32 halo columns each
side as m interleaved words per lane and half-row, the second half mirrored -- and steps it k generations with no
LDS traffic; between blocks the windows of a band swap their edge cells through LDS and the bands hand their k edge
rows to their neighbours as tagged granules.  Bar: bit-exact against the oracle (GameOfLifeLogic.fs:59-63; torus
GameOfLifeDriver.fs:21-25; bounded Script.fsx:6-13) and the BASELINE config-2 golden checkpoints.  Covered: every
window width (m = 3, 5, 9, 17), one window per band (the torus wraps a window onto itself), up to 16 per band, uneven
bands, bands shorter than 2k, depths 1-10, board interleaves 1 / 2 / 4, calls too short for the pass between calls
that take it, the epoch wrap and a timed-out hand-off.  Each case checks that the pass actually ran
("lanes_launches").
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

# gol_last_error() of a timed-out hand-off names its cause and the way out
TIMEOUT_CAUSE = (r"hand-off timed out -- the pass could not get every CU at once \(another process or stream holds "
                 r"the device\); board option \"coop\" 0 avoids the persistent passes")


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _rand(h, w, seed, p=0.45):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


def _run(gol, b0, boundary, steps, m=0, k=None, ilv=0, expect_lanes=True):
    h, w = b0.shape
    opts = {"lanes": 1, "lanes_m": m}
    if k:
        opts["coop_k"] = k
    with gol.Board(w, h, boundary, ilv=ilv, options=opts) as b:
        b.set_cells(b0)
        for g in steps:
            b.step(g)
        assert b.generation == sum(steps)
        ran = b.get_option("lanes_launches")
        assert (ran > 0) == expect_lanes, ran
        return b.get_cells()


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", [(4096, 4096), (1024, 1024), (512, 64), (256, 500), (768, 200), (2048, 300),
                                 (8192, 512), (4096, 37)])
def test_lanes_matches_oracle(gol, oracle, w, h, boundary):
    b0 = _rand(h, w, w + 5 * h + boundary)
    steps = [20, 1, 29]  # blocks of 8 plus remainders; the 1-generation call runs the cooperative pass
    want = oracle.c_run(b0, sum(steps), boundary)
    np.testing.assert_array_equal(_run(gol, b0, boundary, steps), want)


@pytest.mark.parametrize("m", [5, 9, 17])
@pytest.mark.parametrize("boundary", [0, 1])
def test_lanes_window_widths(gol, oracle, m, boundary):
    """Every window width on one board: 4096 wide is 16, 8 or 4 windows of 256, 512 or 1024 columns."""
    b0 = _rand(600, 4096, 11 * m + boundary)
    np.testing.assert_array_equal(_run(gol, b0, boundary, [33], m=m), oracle.c_run(b0, 33, boundary))


@pytest.mark.parametrize("w,m", [(1024, 17), (512, 9), (256, 5)])
def test_lanes_one_window_per_band(gol, oracle, w, m):
    """One window per band: on a torus its left and right halo cells come from its own opposite edge."""
    b0 = _rand(300, w, w + m)
    for boundary in (0, 1):
        np.testing.assert_array_equal(_run(gol, b0, boundary, [40], m=m), oracle.c_run(b0, 40, boundary))


@pytest.mark.parametrize("w", [256, 384, 1024])
def test_lanes_narrow_windows(gol, oracle, w):
    """3 words per lane and half-row: 128-column windows, 2 to 8 per band."""
    b0 = _rand(300, w, 3 * w)
    for boundary in (0, 1):
        np.testing.assert_array_equal(_run(gol, b0, boundary, [33], m=3), oracle.c_run(b0, 33, boundary))


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 10])
def test_lanes_block_depths(gol, oracle, k):
    b0 = _rand(1000, 2048, 50 + k)
    gens = max(2 * k, 23)
    for boundary in (0, 1):
        np.testing.assert_array_equal(_run(gol, b0, boundary, [gens], k=k), oracle.c_run(b0, gens, boundary))


def test_lanes_depth_beyond_window_falls_back(gol, oracle):
    """k = 12 leaves no rows for a band in a 32-row window (32 - 2k < k): the cooperative pass runs instead."""
    b0 = _rand(512, 2048, 3)
    np.testing.assert_array_equal(_run(gol, b0, 0, [40], k=12, expect_lanes=False), oracle.c_run(b0, 40, 0))


@pytest.mark.parametrize("ilv", [1, 2, 4])
def test_lanes_board_interleaves(gol, oracle, ilv):
    """The pass stages any board interleave through LDS as plain words at both ends of a launch."""
    b0 = _rand(400, 8192, 70 + ilv)
    for boundary in (0, 1):
        np.testing.assert_array_equal(_run(gol, b0, boundary, [19], ilv=ilv), oracle.c_run(b0, 19, boundary))


def test_lanes_config2_golden_checkpoints(gol):
    """BASELINE config 2: 4096^2 torus, .NET Random seed 42, every checkpoint to generation 10,000."""
    with open(os.path.join(HERE, "golden", "golden_long.json")) as f:
        case = json.load(f)["c2_4096_torus_dotnet42"]
    with gol.Board(case["width"], case["height"], case["boundary"], options={"lanes": 1}) as b:
        b.seed_dotnet(case["seed"], gol.INIT_DOTNET_MOD2)
        done = 0
        for gen, h, pop in case["checkpoints"]:
            b.step(gen - done)
            done = gen
            assert (b.hash(), b.population()) == (h, pop), gen
        assert b.get_option("lanes_launches") > 0


def test_lanes_epoch_wrap(gol, oracle):
    b0 = _rand(1024, 1024, 78)
    with gol.Board(1024, 1024, 0, options={"lanes": 1}) as b:
        b.set_cells(b0)
        b.step(23)  # >= 2 blocks of this width's depth (10)
        done = 23
        for epoch in (0xfffd, 0xfffe, 0xffff):
            b.set_option("coop_epoch", epoch)
            b.step(23)
            done += 23
        b.step(23)
        done += 23
        assert b.get_option("lanes_launches") == 5
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, done, 0))


def test_lanes_timeout_reported(gol, oracle):
    """A hand-off wait that times out (a one-poll spin limit) leaves a wrong board; readbacks report it, the
    launch ends, and the board is usable again once overwritten."""
    b0 = _rand(2048, 2048, 93)
    with gol.Board(2048, 2048, 0, options={"lanes": 1, "coop_k": 1, "coop_spin_limit": 1,
                                           "coop_poll_delay": 0}) as b:
        b.set_cells(b0)
        failed = False
        for _ in range(20):
            b.step(200)
            try:
                b.synchronize()
            except RuntimeError:
                failed = True
                break
        assert failed, "a one-poll spin limit never timed out"
        with pytest.raises(RuntimeError, match=TIMEOUT_CAUSE):
            b.get_cells()
        b.set_option("coop_spin_limit", 0)
        b.set_cells(b0)
        b.step(37)
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 37, 0))
