"""Independent handles under the persistent passes, and boards the rows-on-lanes pass cannot hold resident.

* the cooperative and rows-on-lanes passes are persistent grids whose bands spin on each
  other; two such grids resident together could split the CUs and starve both.  The library serialises persistent
  launches per device (csrc/gol_coop.hip launch_persistent), so two handles stepped from two threads at once -- the
  reference's timer and render threads may drive the engine concurrently, GameOfLifeDriver.fs:38-40,
  GameOfLifeUI.fs:29-31; gol.h promises independent handles -- both finish exact.
* a tall narrow packed board plans more lanes bands than the device holds at once; such a
  board must fall through to the cooperative or the streaming pass instead of failing the launch.
"""
import json
import os
import threading

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


def test_two_handles_two_threads_persistent_passes(gol):
    """Two 4096^2 handles (BASELINE config 2, .NET Random seed 42), one on the cooperative pass and one on the
    rows-on-lanes pass, each stepped 1000 generations from its own thread at the same time: both match the golden
    checkpoint at generation 1000 (tests/golden/golden_long.json c2_4096_torus_dotnet42), no GOL_ERR_HIP."""
    with open(os.path.join(HERE, "golden", "golden_long.json")) as f:
        case = json.load(f)["c2_4096_torus_dotnet42"]
    want = {gen: (h, pop) for gen, h, pop in case["checkpoints"]}[1000]
    boards = [gol.Board(case["width"], case["height"], case["boundary"], options={"coop": 1, "lanes": lanes})
              for lanes in (0, 1)]
    try:
        for b in boards:
            b.seed_dotnet(case["seed"], gol.INIT_DOTNET_MOD2)
        start = threading.Barrier(2)
        results, errors = [None, None], []

        def drive(i):
            try:
                start.wait()
                for _ in range(10):  # ten calls of 100 generations: launches of both boards interleave
                    boards[i].step(100)
                results[i] = (boards[i].hash(), boards[i].population())
            except Exception as e:  # reported below, on the main thread
                errors.append(e)

        threads = [threading.Thread(target=drive, args=(i,)) for i in range(2)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in threads), "a board did not finish"
        assert not errors, errors
        assert results[0] == want and results[1] == want
        assert boards[0].get_option("lanes_launches") == 0 and boards[1].get_option("lanes_launches") == 10
    finally:
        for b in boards:
            b.close()


@pytest.mark.parametrize("w,h", [(1024, 16384), (256, 65536)])
def test_tall_narrow_packed_board(gol, oracle, w, h):
    """Packed boards whose rows-on-lanes plan has more bands than the device holds (1024 x 16384: 1366 bands of 8
    waves; 256 x 65536: 5462 bands of 2 waves) run on another pass, exact against the oracle."""
    b0 = (np.random.default_rng(w + h).random((h, w)) < 0.4).astype(np.uint8)
    with gol.Board(w, h, 0) as b:
        assert b.info()["packed"]
        b.set_cells(b0)
        b.step(24)
        assert b.get_option("lanes_launches") == 0
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 24, 0))
