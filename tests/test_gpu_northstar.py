"""The north-star claim at full size (BASELINE.json: "bit-exact boards versus the reference after 10k
generations ... on a 65536^2 and larger board"; configs 3 and 4).

Every checkpoint of tests/golden/golden_full.json -- the CPU oracle's bit-packed stepper (oracle/gol_fast.c,
pinned to the byte-per-cell oracle in tests/test_oracle.py) run on the same splitmix-seeded boards -- is
compared (canonical hash + population) with three GPU paths, each applying the rule of
GameOfLifeLogic.fs:59-63 once per tick of GameOfLifeDriver.fs:32-40:

  * the shipped single board (gol_create defaults: M = 2, K = 12 in 12-wave workgroups on both boundaries since
    round 3; the bounded K = 16 pass keeps its own full-size case) -- the kernel bench.py times;
  * 8 ghost-row strips driven by one process (strips.LocalBoard): the per-rank kernel and halo geometry of
    the torchrun/RCCL bench path;
  * the one-handle multi-GPU board (gol_create_multi, 8 strips, peer-copied halos: csrc/gol_multi.cpp),
    what the F# drop-in calls, with every strip on device 0 of the one-GPU box.
"""
import json
import os

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FULL = os.path.join(HERE, "golden", "golden_full.json")


def _cases():
    if not os.path.exists(FULL):
        return {}
    with open(FULL) as f:
        return json.load(f)


def _case(name):
    c = _cases().get(name)
    if c is None:
        pytest.skip(f"{name} not in golden_full.json (tests/golden/make_golden_full.py)")
    return c


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _free_torch_cache():
    import torch

    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _walk(board, case, step, observe):
    """Advance through every checkpoint, comparing (hash, population)."""
    done = 0
    for gen, h, pop in case["checkpoints"]:
        if gen > done:
            step(gen - done)
            done = gen
        got = observe()
        assert got == (h, pop), f"generation {gen}: got {got}, oracle {(h, pop)}"


@pytest.mark.parametrize("name", ["n1_65536_torus", "n1_65536_bounded", "c4_262144_torus"])
def test_single_board_shipped_defaults(gol, name):
    c = _case(name)
    with gol.Board(c["width"], c["height"], c["boundary"]) as b:
        info = b.info()
        # the level-pipelined pass on both boundaries (round 6)
        want = (4, 32)
        assert (info["ilv"], info["tblock_k"]) == want
        b.seed_splitmix(c["seed"])
        _walk(b, c, b.step, lambda: (b.hash(), b.population()))
        assert b.generation == c["generations"]


def test_single_board_bounded_k16(gol):
    """The bounded board on the streaming pass at K = 16 (its default before round 3, still the depth of mid-size
    boards; round 6 moved the default to the level-pipelined pass)."""
    c = _case("n1_65536_bounded")
    with gol.Board(c["width"], c["height"], c["boundary"], tblock_k=16, ilv=2) as b:
        assert b.info()["tblock_k"] == 16
        b.seed_splitmix(c["seed"])
        _walk(b, c, b.step, lambda: (b.hash(), b.population()))


@pytest.mark.parametrize("name", ["n1_65536_torus", "c4_262144_torus"])
def test_ghost_row_strips_8(gol, name):
    import torch

    from gameoflifewithactors_amd.strips import LocalBoard

    c = _case(name)
    lb = LocalBoard(c["width"], c["height"], c["boundary"], 12, 8)
    try:
        lb.seed_splitmix(c["seed"])
        _walk(lb, c, lb.step, lambda: (lb.hash(), lb.population()))
    finally:
        del lb
        _free_torch_cache()
    assert torch.cuda.current_device() == 0


@pytest.mark.parametrize("name", ["n1_65536_torus", "n1_65536_bounded", "c4_262144_torus"])
def test_multi_gpu_handle_8_strips(gol, name):
    c = _case(name)
    with gol.Board(c["width"], c["height"], c["boundary"], devices=[0] * 8) as b:
        assert len(b.parts()) == 8
        b.seed_splitmix(c["seed"])
        _walk(b, c, b.step, lambda: (b.hash(), b.population()))
