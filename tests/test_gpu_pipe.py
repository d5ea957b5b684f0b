"""GPU parity of the level-pipelined deep pass (csrc/gol_pipe.hip).

A torus board at ilv 4 with K = 16 or 32 runs this pass: each of a strip's K levels is held by one of S waves of D = 4
levels, rows handed between the waves through LDS rings.  Bar: bit-exact against the oracle (rule
GameOfLifeLogic.fs:59-63, torus GameOfLifeDriver.fs:21-25) on every column geometry the planner makes -- full strips
only, one strip plus remainder sub-strips packed 1 to 21 per wave, a remainder wide enough to become an overlapping
strip -- on heights that leave short and empty pipelines, at every pipeline share (board option "pipe_split"), on the
ghost-row strips of the multi-GPU path, and at the north-star size against the committed golden checkpoints.  Every
test also checks the library's error word of the pass (a ring wait that gave up) is clear.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _pipe_errors():
    import ctypes

    from gameoflifewithactors_amd import _lib

    v = ctypes.c_int()
    assert _lib.load().gol_debug_pipe_errors(ctypes.byref(v)) == 0
    return v.value


def _rand(h, w, seed, p=0.4):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


def _run(gol, b0, k, gens, opts=None, boundary=0):
    h, w = b0.shape
    with gol.Board(w, h, boundary, tblock_k=k, ilv=4, options=dict(opts or {}, coop=0)) as b:
        assert b.info()["tblock_k"] == k and b.info()["ilv"] == 4
        b.set_cells(b0).step(gens)
        return b.get_cells()


@pytest.mark.parametrize("k", [16, 32])
@pytest.mark.parametrize("nblocks,h", [
    (62, 203),    # one full strip, no remainder
    (64, 300),    # one strip + 2 blocks: 16 sub-strips of 4 lanes per remainder wave
    (65, 97),     # + 3 blocks: 12 sub-strips
    (80, 257),    # + 18 blocks: 3 sub-strips of 20 lanes
    (92, 129),    # + 30 blocks: 2 sub-strips of 32 lanes
    (94, 150),    # + 32 blocks: one more strip, overlapping the last full one
    (125, 333),   # 2 strips + 1 block: 21 sub-strips of 3 lanes
    (140, 41),    # fewer rows than the 2K-row cone: most pipelines empty
])
def test_pipe_matches_oracle(gol, oracle, k, nblocks, h):
    w = 128 * nblocks
    b0 = _rand(h, w, nblocks * 131 + h + k)
    gens = 2 * k + 5  # two pipelined passes, then the streaming pass at ilv 4 for the last 5
    want = oracle.c_run(b0, gens, 0)
    np.testing.assert_array_equal(_run(gol, b0, k, gens), want)
    assert _pipe_errors() == 0


@pytest.mark.parametrize("k", [16, 32])
@pytest.mark.parametrize("nblocks,h", [
    (64, 203),    # one strip: both board edges on the wave's outer lanes
    (65, 97),     # two edge strips, overlapping by 62 blocks
    (126, 300),   # two edge strips meeting exactly
    (127, 129),   # two edge strips and 1 remainder block between them (21 sub-strips per wave)
    (140, 257),   # 14 remainder blocks (4 sub-strips per wave, packed over row groups)
    (157, 150),   # a remainder of 31 blocks: one more strip instead, overlapping
    (200, 41),    # 3 strips + 12 blocks; fewer rows than the 2K-row cone: every group reaches past both board edges
])
def test_pipe_bounded_matches_oracle(gol, oracle, k, nblocks, h):
    """Bounded boards (Script.fsx:6-13: dead beyond the edges) on the pass: strips of 64 blocks with the board's
    edges on a wave's outer lanes (zero-filled lane moves), remainder sub-strips between the last two, rows outside the
    board loaded as zeros and kept dead at every level, against the oracle."""
    w = 128 * nblocks
    b0 = _rand(h, w, nblocks * 7 + h + k)
    gens = 2 * k + 5
    np.testing.assert_array_equal(_run(gol, b0, k, gens, boundary=1), oracle.c_run(b0, gens, 1))
    assert _pipe_errors() == 0


def test_pipe_bounded_live_edges(gol, oracle):
    """Cells alive on all four edges of a bounded board: births just outside the board must never happen (a glider
    leaving through a corner, full edge rows and columns), on the pass against the oracle."""
    w, h, k = 128 * 65, 150, 32
    b0 = np.zeros((h, w), np.uint8)
    b0[0, :] = 1
    b0[-1, :] = 1
    b0[:, 0] = 1
    b0[:, -1] = 1
    b0[1:4, 1:4] = [[0, 1, 0], [0, 0, 1], [1, 1, 1]]
    b0[60:63, w - 3:w] = [[1, 1, 1], [0, 0, 1], [0, 1, 0]]
    gens = 3 * k + 1
    np.testing.assert_array_equal(_run(gol, b0, k, gens, boundary=1), oracle.c_run(b0, gens, 1))
    assert _pipe_errors() == 0


def test_pipe_bounded_ghost_row_strips(gol, oracle):
    """The multi-GPU rank kernel on a bounded board: 3 ghost-row strips (the end strips' outer ghost rows beyond the
    board, dead), against the oracle."""
    import torch

    from gameoflifewithactors_amd.strips import LocalBoard

    w, h, k = 128 * 66, 700, 32
    b0 = _rand(h, w, 23)
    with LocalBoard(w, h, 1, k, 3, ilv=4) as lb:
        assert all(r.geom.ilv == 4 and r.geom.ghost == k for r in lb.runners)
        lb.set_cells(torch.as_tensor(b0))
        lb.step(3 * k + 8)
        np.testing.assert_array_equal(lb.get_cells().numpy(), oracle.c_run(b0, 3 * k + 8, 1))
    assert _pipe_errors() == 0


@pytest.mark.parametrize("split", [-1, int(0.55 * 65536), int(0.8 * 65536)])
def test_pipe_shares_do_not_change_results(gol, oracle, split):
    """The pipelines' row shares (board option "pipe_split": equal, and two age ratios) move rows between the
    pipelines of a workgroup, never the result."""
    w, h, k = 128 * 64, 700, 32
    b0 = _rand(h, w, split & 0xffff)
    want = oracle.c_run(b0, 2 * k, 0)
    np.testing.assert_array_equal(_run(gol, b0, k, 2 * k, {"pipe_split": split, "pipe_split2": split}), want)


def test_pipe_ghost_row_strips(gol, oracle):
    """The multi-GPU rank kernel on this pass: 3 ghost-row strips (gol_strip_step, K ghost rows) in one process,
    interior launches leaving room for the edge bands (spare waves), against the oracle."""
    import torch

    from gameoflifewithactors_amd.strips import LocalBoard

    w, h, k = 128 * 70, 900, 32
    b0 = _rand(h, w, 11)
    with LocalBoard(w, h, 0, k, 3, ilv=4) as lb:
        assert all(r.geom.ilv == 4 and r.geom.ghost == k for r in lb.runners)
        lb.set_cells(torch.as_tensor(b0))
        lb.step(3 * k + 8)
        np.testing.assert_array_equal(lb.get_cells().numpy(), oracle.c_run(b0, 3 * k + 8, 0))
    assert _pipe_errors() == 0


@pytest.mark.parametrize("w,h,boundary", [(128 * 63, 300, 1), (128 * 61, 300, 0), (512, 96, 0)])
def test_pipe_depth_is_a_cap_where_the_pass_does_not_run(gol, oracle, w, h, boundary):
    """tblock_k is a cap (gol.h): at ilv 4 the depths 16 / 32 are the level-pipelined pass, which runs on torus rows
    holding a full strip of 62 blocks and bounded rows of at least 64; a narrower board asked for them runs the
    streaming pass's deepest ilv-4 depth (8) instead, exact against the oracle, and a strip pass asked for them is
    refused."""
    import ctypes

    from gameoflifewithactors_amd import _lib

    b0 = _rand(h, w, w + h + boundary)
    gens = 37
    with gol.Board(w, h, boundary, tblock_k=32, ilv=4, options={"coop": 0}) as b:
        b.set_cells(b0).step(gens)
        got = b.get_cells()
    np.testing.assert_array_equal(got, oracle.c_run(b0, gens, boundary))
    lib = _lib.load()
    s = _lib.Strip(w, h, 0, h, 0, w // 32, boundary, 1 if boundary == 0 else 0, 4, 0)
    rc = lib.gol_strip_step(ctypes.byref(s), ctypes.c_void_p(16), ctypes.c_void_p(32), 16, 0, h, None)
    assert rc == -1 and b"level-pipelined" in lib.gol_last_error()


def _golden(name):
    path = os.path.join(HERE, "golden", "golden_full.json")
    if not os.path.exists(path):
        pytest.skip("no golden_full.json")
    with open(path) as f:
        c = json.load(f).get(name)
    if c is None:
        pytest.skip(f"{name} not in golden_full.json")
    return c


def test_pipe_northstar_board_defaults(gol):
    """The north-star board (65536^2 torus, splitmix seed) on the shipped defaults is this pass (ilv 4, K = 32) and
    matches the oracle's checkpoints to generation 2000 (tests/test_gpu_northstar.py walks all 10,000)."""
    c = _golden("n1_65536_torus")
    with gol.Board(c["width"], c["height"], c["boundary"]) as b:
        assert (b.info()["ilv"], b.info()["tblock_k"]) == (4, 32)
        b.seed_splitmix(c["seed"])
        done = 0
        for gen, h, pop in c["checkpoints"]:
            if gen > 2000:
                break
            b.step(gen - done)
            done = gen
            assert (b.hash(), b.population()) == (h, pop), f"generation {gen}"
    assert _pipe_errors() == 0


def test_pipe_northstar_as_two_ghost_strips(gol):
    """65536^2 as two ghost-row strips of 32768 rows (2^31 cells each: an N = 2 rank's pipelined pass) in one
    process, against the oracle's generation-1000 checkpoint."""
    import torch

    from gameoflifewithactors_amd.strips import LocalBoard

    c = _golden("n1_65536_torus")
    gen, h, pop = next(x for x in c["checkpoints"] if x[0] == 1000)
    with LocalBoard(c["width"], c["height"], 0, 32, 2, ilv=4) as lb:
        lb.seed_splitmix(c["seed"])
        lb.step(gen)
        assert (lb.hash(), lb.population()) == (h, pop)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    assert _pipe_errors() == 0
