"""GPU tests of the row-strip path (gol_strip_* kernels with ghost rows) on one device: N strips of one
board driven in-process (strips.LocalBoard, device-to-device halo copies) must equal the oracle and
the single-board path bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nstrips", [2, 3, 4])
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("k", [1, 4, 8])
@pytest.mark.parametrize("ilv", [1, 2, 4])
def test_local_strips_match_oracle(oracle, nstrips, boundary, k, ilv):
    from gameoflifewithactors_amd.strips import LocalBoard

    w, h, gens = {1: 96, 2: 320, 4: 256}[ilv], 4 * 16 + 7, 41
    b0 = (np.random.default_rng(nstrips * 10 + k).random((h, w)) < 0.45).astype(np.uint8)
    lb = LocalBoard(w, h, boundary, k, nstrips)
    lb.set_cells(b0)
    lb.step(gens)
    want = oracle.c_run(b0, gens, boundary)
    assert np.array_equal(lb.get_cells().numpy(), want)
    assert lb.hash() == oracle.board_hash(want)


def test_local_strips_large_match_single_board():
    from gameoflifewithactors_amd import Board
    from gameoflifewithactors_amd.strips import LocalBoard

    w, h, gens, seed = 65536, 4096, 64, 99
    with Board(w, h, tblock_k=8) as b:
        b.seed_splitmix(seed)
        b.step(gens)
        want = b.hash()
    lb = LocalBoard(w, h, 0, 8, 4)
    lb.seed_splitmix(seed)
    lb.step(gens)
    assert lb.hash() == want


def test_strip_runner_single_rank_matches_board():
    from gameoflifewithactors_amd import Board
    from gameoflifewithactors_amd.strips import StripRunner

    for boundary in (0, 1):
        r = StripRunner(4096, 1000, boundary, 8, device=torch.device("cuda", 0))
        r.seed_splitmix(5)
        r.step(100)
        with Board(4096, 1000, boundary, tblock_k=8) as b:
            b.seed_splitmix(5).step(100)
            assert r.hash() == b.hash() and r.population() == b.population()
