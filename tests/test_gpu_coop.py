"""GPU parity of the cooperative register-band pass for mid-size boards (csrc/gol_coop.hip).

Packed boards above the LDS-resident cut-over (2^17 cells), up to 2^25 cells and 8192 wide, run every gol_step
call as one persistent launch: one workgroup per CU holds a band of rows in registers, exchanges wave-edge
rows through LDS every generation and hands its K edge rows to its two neighbour bands every K generations.
Bar: bit-exact against the oracle (GameOfLifeLogic.fs:59-63; torus GameOfLifeDriver.fs:21-25; bounded
Script.fsx:6-13), the BASELINE config-2 golden checkpoints (4096^2, .NET Random seed 42, 10k generations), and
the streaming pass on the same board (board option "coop" 0).  Uneven bands (heights that do not divide over the CUs),
bands shorter than two blocks, several block depths ("coop_k"), both word layouts (consecutive words of an
ilv-1 board, interleaved blocks of an ilv-2 / ilv-4 board), ragged byte boards (widths not a multiple of 32,
through whole-word scratch rows) and split calls are covered.
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


def _run(gol, b0, boundary, steps, coop, k=None, ilv=0):
    h, w = b0.shape
    opts = {"coop": int(coop), "lanes": 0}
    if k:
        opts["coop_k"] = k
    with gol.Board(w, h, boundary, ilv=ilv, options=opts) as b:
        if not ilv:  # single boards of the widths the pass holds interleaved get its layout, on either path
            assert b.info()["ilv"] == (w // 2048 if w in (4096, 8192) else 1)
        b.set_cells(b0)
        for g in steps:
            b.step(g)
        assert b.generation == sum(steps)
        return b.get_cells()


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", [(1024, 1024), (512, 2048), (2048, 300), (4096, 4096), (2016, 1500), (8192, 512)])
def test_coop_matches_oracle_and_streaming(gol, oracle, w, h, boundary):
    b0 = _rand(h, w, w + 3 * h + boundary)
    steps = [1, 20, 0, 29]  # split calls; blocks of 8 plus remainders
    want = oracle.c_run(b0, sum(steps), boundary)
    np.testing.assert_array_equal(_run(gol, b0, boundary, steps, coop=True), want)
    np.testing.assert_array_equal(_run(gol, b0, boundary, steps, coop=False), want)


@pytest.mark.parametrize("w,h", [(4096, 700), (8192, 300), (2048, 1024)])
def test_coop_consecutive_words(gol, oracle, w, h):
    """An ilv-1 board of a width the pass holds as 2 or 4 consecutive words per lane."""
    b0 = _rand(h, w, w + h)
    for boundary in (0, 1):
        want = oracle.c_run(b0, 21, boundary)
        np.testing.assert_array_equal(_run(gol, b0, boundary, [21], coop=True, ilv=1), want)


@pytest.mark.parametrize("k", [1, 3, 8, 16])
def test_coop_block_depths(gol, oracle, k):
    b0 = _rand(1024, 2048, 40 + k)
    for boundary in (0, 1):
        np.testing.assert_array_equal(_run(gol, b0, boundary, [37], coop=True, k=k), oracle.c_run(b0, 37, boundary))


def test_coop_config2_golden_checkpoints(gol):
    """BASELINE config 2: 4096^2 torus, .NET Random seed 42 in the reference's order, every checkpoint (hash +
    population every 100 generations) to generation 10,000, on the cooperative pass."""
    with open(os.path.join(HERE, "golden", "golden_long.json")) as f:
        case = json.load(f)["c2_4096_torus_dotnet42"]
    with gol.Board(case["width"], case["height"], case["boundary"], options={"coop": 1, "lanes": 0}) as b:
        b.seed_dotnet(case["seed"], gol.INIT_DOTNET_MOD2)
        done = 0
        for gen, h, pop in case["checkpoints"]:
            b.step(gen - done)
            done = gen
            assert (b.hash(), b.population()) == (h, pop), gen


def test_coop_epoch_wrap(gol, oracle):
    """The hand-off granules carry a 16-bit launch epoch; at the wrap the host clears them. Launches just before,
    at and after the wrap (the "coop_epoch" option sets the epoch of the last launch) must stay exact."""
    b0 = _rand(1024, 1024, 77)
    with gol.Board(1024, 1024, 0, options={"coop": 1, "lanes": 0}) as b:
        b.set_cells(b0)
        b.step(9)  # first launch: allocates and clears the exchange buffer
        done = 9
        for epoch in (0xfffd, 0xfffe, 0xffff):
            b.set_option("coop_epoch", epoch)
            b.step(17)  # this launch runs at epoch + 1 (the last one wraps to 1 and clears)
            done += 17
        b.step(17)
        done += 17
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, done, 0))


@pytest.mark.parametrize("lanes", [0, 1])
def test_epoch_set_back_reuses_no_stale_granule(gol, oracle, lanes):
    """the debug knob "coop_epoch" set to the last launch's epoch - 1 makes the next launch
    run at the SAME epoch as the last one, whose granules (block 0 of parity 0 included) are still in the exchange
    buffer.  Setting the epoch clears the buffer, so the launch must poll for its own neighbours' data and stay
    exact.  4096^2, 16 generations after the reuse, on the cooperative and the rows-on-lanes pass."""
    b0 = _rand(4096, 4096, 95)
    with gol.Board(4096, 4096, 0, options={"coop": 1, "lanes": lanes}) as b:
        b.set_cells(b0)
        b.step(16)
        last = b.get_option("coop_epoch")
        b.set_option("coop_epoch", last - 1)
        b.step(16)
        assert b.get_option("coop_epoch") == last
        if lanes:
            assert b.get_option("lanes_launches") == 2
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 32, 0))


def test_debug_knobs_are_not_board_options(gol):
    """gol.h's option list holds only product settings: the test knobs are refused by gol_set_option /
    gol_get_option and reached through gol_debug_set_option (csrc/gol_debug.h)."""
    import ctypes

    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    with gol.Board(1024, 1024, 0) as b:
        v = ctypes.c_int64()
        for name in sorted(_lib.DEBUG_OPTIONS):
            assert lib.gol_set_option(b._h, name.encode(), 1) == _lib.GOL_ERR_INVALID, name
            assert lib.gol_get_option(b._h, name.encode(), ctypes.byref(v)) == _lib.GOL_ERR_INVALID, name
            assert lib.gol_debug_get_option(b._h, name.encode(), ctypes.byref(v)) == _lib.GOL_OK, name
        for name in ("coop", "coop_k", "lanes", "split"):
            assert lib.gol_debug_set_option(b._h, name.encode(), 0) == _lib.GOL_ERR_INVALID, name


@pytest.mark.parametrize("w,h", [(2048, 2048), (4096, 1024), (8192, 512)])
def test_coop_timeout_reported_on_every_readback(gol, oracle, w, h):
    """A band hand-off wait that times out (forced here: a spin limit of one poll, while the neighbour band has not
    published yet) leaves a wrong board.  Every readback and gol_synchronize must report it (GOL_ERR_HIP), the
    launch must still end (no further waits once one has failed), and the board must be usable again once it is
    overwritten.  Round 5: on each hand-off form -- 8-byte granules (M = 1), 16-byte pairs (M = 2),
    and the 256-word rows that read the error word before polling (M = 4)."""
    b0 = _rand(h, w, 91)
    with gol.Board(w, h, 0, options={"coop": 1, "lanes": 0, "coop_k": 1, "coop_spin_limit": 1, "coop_poll_delay": 0}) as b:
        b.set_cells(b0)
        failed = False
        for _ in range(20):  # the race is lost almost always at once; a few tries make it certain
            b.step(200)
            try:
                b.synchronize()
            except RuntimeError:
                failed = True
                break
        assert failed, "a one-poll spin limit never timed out"
        for call in (b.get_cells, b.hash, b.population, b.save_packed, lambda: b.get_region(0, 0, 8, 8),
                     b.synchronize):
            with pytest.raises(RuntimeError, match=TIMEOUT_CAUSE):
                call()
        b.set_option("coop_spin_limit", 0)  # back to the default limit
        b.set_cells(b0)  # overwritten: valid again
        b.step(37)
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 37, 0))


def test_coop_timeout_then_overwrite_without_readback(gol, oracle):
    """a cooperative pass that timed out, with NO readback or gol_synchronize after it, then an
    overwrite: the overwrite must succeed (the stale error word is cleared without marking the board invalid) and
    the board must read back valid and exact."""
    b0 = _rand(2048, 2048, 92)
    with gol.Board(2048, 2048, 0, options={"coop": 1, "lanes": 0, "coop_k": 1, "coop_spin_limit": 1, "coop_poll_delay": 0}) as b:
        b.set_cells(b0)
        for _ in range(5):  # nothing reads the error word in between
            b.step(200)
        b.set_option("coop_spin_limit", 0)
        for overwrite in (lambda: b.set_cells(b0), lambda: b.load_packed(oracle.pack64(b0)),
                          lambda: b.seed_splitmix(3) and b.set_cells(b0)):
            b.set_option("coop_spin_limit", 1)
            b.step(200)
            b.set_option("coop_spin_limit", 0)
            overwrite()  # must not raise
            b.step(37)
            np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 37, 0))


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", [(129, 300), (1001, 257), (2047, 90), (2049, 131), (4095, 64), (4097, 77),
                                 (8191, 40), (333, 1000)])
def test_coop_ragged_widths(gol, oracle, w, h, boundary):
    """Byte boards of widths that are not a multiple of 32 and that the single-wave pass does not take run on
    the cooperative pass through whole-word scratch rows (calls of >= 16 generations), with the row end patched
    at bit level: torus wrap from cell W - 1 to cell 0 (GameOfLifeDriver.fs:21-25), dead beyond both ends when
    bounded (Script.fsx:6-13).  Rows of 1, 2 and 4 words per lane, padded rows (2049, 4097), split calls and a
    remainder block, against the oracle and against the per-generation byte step ("coop" 0)."""
    b0 = _rand(h, w, w + 7 * h + boundary)
    steps = [16, 3, 21]  # 3 < 16: the byte step between two pass calls
    want = oracle.c_run(b0, sum(steps), boundary)
    for coop in (True, False):
        with gol.Board(w, h, boundary, options={"coop": int(coop), "lanes": 0}) as b:
            assert not b.info()["packed"]
            b.set_cells(b0)
            for g in steps:
                b.step(g)
            assert b.generation == sum(steps)
            np.testing.assert_array_equal(b.get_cells(), want, err_msg=f"coop={coop}")


def test_coop_ragged_byte_values(gol, oracle):
    """Byte cells are alive when nonzero (any value); the ragged pass writes the board back as 0 / 1."""
    b0 = _rand(200, 1001, 5)
    vals = (b0 * np.random.default_rng(6).integers(1, 256, size=b0.shape)).astype(np.uint8)
    with gol.Board(1001, 200, 0, options={"coop": 1, "lanes": 0}) as b:
        b.set_cells(vals)
        b.step(24)
        np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 24, 0))
