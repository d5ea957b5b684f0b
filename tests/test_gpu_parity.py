"""GPU parity tests: the HIP path (through the C ABI, libgol_hip.so) against the CPU oracle.

Bar: bit-exact boards (integer work).  Oracle = oracle/gol_oracle.{c,py} (test infrastructure).
Sizes are chosen so the oracle finishes in seconds; full-size boards are checked through
size-independent properties (windowed light-cone checks against the oracle, temporal-block
invariance, hash/population consistency).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KS = [1, 2, 4, 6, 8, 12, 16, 24, 32]  # caps: each layout uses its deepest supported depth <= k


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _rand(h, w, seed, p=0.5):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


# ---------------------------------------------------------------- small boards vs the oracle
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("ilv", [1, 2, 4])
@pytest.mark.parametrize("w,h", [(32, 3), (64, 5), (96, 64), (128, 127), (320, 77), (2048, 40), (4000 + 96, 9)])
def test_packed_step_matches_oracle(gol, oracle, boundary, ilv, w, h):
    if w % (32 * ilv):
        pytest.skip("width is not a whole number of blocks for this layout")
    b0 = _rand(h, w, w * 1000 + h)
    want = {1: oracle.c_run(b0, 1, boundary)}
    want[37] = oracle.c_run(want[1], 36, boundary)
    for k in KS:
        with gol.Board(w, h, boundary, tblock_k=k, ilv=ilv) as b:
            assert b.info()["packed"] and b.info()["ilv"] == ilv
            b.set_cells(b0)
            assert np.array_equal(b.get_cells(), b0)
            b.step(1)
            assert np.array_equal(b.get_cells(), want[1]), f"k={k} gen 1"
            b.step(36)
            assert np.array_equal(b.get_cells(), want[37]), f"k={k} gen 37"


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h", [(3, 3), (100, 100), (33, 7), (257, 40), (181, 181), (1001, 33), (333, 333)])
def test_byte_path_matches_oracle(gol, oracle, boundary, w, h):
    """Ragged widths (byte-per-cell board, one gol_bytes_step launch per generation), split step calls."""
    b0 = _rand(h, w, w + 7 * h)
    with gol.Board(w, h, boundary) as b:
        assert not b.info()["packed"]
        b.set_cells(b0)
        b.step(25)
        assert np.array_equal(b.get_cells(), oracle.c_run(b0, 25, boundary))
        b.step(1)
        b.step(4)
        assert b.generation == 30
        assert np.array_equal(b.get_cells(), oracle.c_run(b0, 30, boundary))


@pytest.mark.parametrize("k", KS)
@pytest.mark.parametrize("ilv", [1, 2, 4])
def test_deep_pass_matches_oracle_many_generations(gol, oracle, k, ilv):
    """One long run (K-blocked passes + remainder passes) against 150 oracle generations."""
    b0 = _rand(96, 256, 99 + k, p=0.35)
    for boundary in (0, 1):
        with gol.Board(256, 96, boundary, tblock_k=k, ilv=ilv) as b:
            b.set_cells(b0).step(150)
            assert np.array_equal(b.get_cells(), oracle.c_run(b0, 150, boundary))


def test_edge_cases(gol, oracle):
    for boundary in (0, 1):
        with gol.Board(64, 64, boundary) as b:  # empty board stays empty
            b.step(100)
            assert b.population() == 0
        full = np.ones((8, 64), np.uint8)
        with gol.Board(64, 8, boundary) as b:
            b.set_cells(full).step(1)
            assert np.array_equal(b.get_cells(), oracle.c_run(full, 1, boundary))
    with gol.Board(64, 64) as b:
        b.step(0)
        assert b.generation == 0


# ---------------------------------------------------------------- golden fixtures
def _golden():
    with open(os.path.join(HERE, "golden", "golden_small.json")) as f:
        return json.load(f)["cases"]


def _setup(gol, b, case, oracle):
    if case["init"] == "dotnet-mod2":
        b.seed_dotnet(case["seed"], gol.INIT_DOTNET_MOD2)
    elif case["init"] == "dotnet-next2":
        b.seed_dotnet(case["seed"], gol.INIT_DOTNET_NEXT2)
    elif case["init"] == "splitmix":
        b.seed_splitmix(case["seed"])
    else:
        pats = {"gosper_gun": oracle.GOSPER_GUN, "r_pentomino": oracle.R_PENTOMINO}
        for name, x, y in case["rle"]:
            b.place_rle(pats[name], x, y)


@pytest.mark.parametrize("name", sorted(_golden()))
@pytest.mark.parametrize("k", [1, 16])
def test_golden_fixtures(gol, oracle, name, k):
    case = _golden()[name]
    boards = np.load(os.path.join(HERE, "golden", "golden_boards.npz"))
    bd = 0 if case["boundary"] == "torus" else 1
    w, h = case["width"], case["height"]
    with gol.Board(w, h, bd, tblock_k=k) as b:
        _setup(gol, b, case, oracle)
        done = 0
        for cp in sorted(int(c) for c in case["checkpoints"]):
            b.step(cp - done)
            done = cp
            want = case["checkpoints"][str(cp)]
            assert str(b.hash()) == want["hash"], f"{name} gen {cp}"
            assert b.population() == want["population"]
            key = f"{name}_g{cp}"
            if key in boards.files:
                got = np.packbits(b.get_cells(), axis=None, bitorder="little")
                assert np.array_equal(got, boards[key])


# ---------------------------------------------------------------- observables / formats
def test_hash_population_render_region(gol, oracle):
    b0 = _rand(50, 320, 5)
    with gol.Board(320, 50) as b:
        b.set_cells(b0)
        assert b.hash() == oracle.board_hash(b0)
        assert b.population() == oracle.population(b0)
        assert np.array_equal(b.render_gray8(128), oracle.render_gray8(b0, 128))
        assert np.array_equal(b.render_gray8(255, stride=333), oracle.render_gray8(b0, 255, stride=333))
        assert np.array_equal(b.get_region(17, 3, 100, 20), b0[3:23, 17:117])
    with gol.Board(100, 30) as b:  # byte path
        b0 = _rand(30, 100, 6)
        b.set_cells(b0)
        assert b.hash() == oracle.board_hash(b0) and b.population() == oracle.population(b0)
        assert np.array_equal(b.render_gray8(128), oracle.render_gray8(b0, 128))


@pytest.mark.parametrize("w,h", [(100, 100), (128, 64), (333, 9)])
def test_seeding_matches_oracle(gol, oracle, w, h):
    with gol.Board(w, h) as b:
        for mode in (0, 1):
            b.seed_dotnet(42, mode)
            assert np.array_equal(b.get_cells(), oracle.seed_dotnet(w, h, 42, mode))
        b.seed_splitmix(0x5EED)
        assert np.array_equal(b.get_cells(), oracle.seed_splitmix(w, h, 0x5EED))


def test_place_rle_wraps(gol, oracle):
    with gol.Board(64, 64) as b:
        b.place_rle(oracle.GOSPER_GUN, 50, 60)
        want = oracle.place_rle(np.zeros((64, 64), np.uint8), oracle.GOSPER_GUN, 50, 60)
        assert np.array_equal(b.get_cells(), want)
    with gol.Board(64, 64) as b, pytest.raises(ValueError):
        b.place_rle("3o?", 0, 0)


# ---------------------------------------------------------------- known answers at larger sizes
def test_glider_period_on_large_torus(gol, oracle):
    w = 4096
    with gol.Board(w, 64) as b:
        b.place_rle(oracle.GLIDER, 100, 20)
        h0 = b.hash()
        b.step(4 * 64)  # vertical period 4H moves it 64 cells right, not yet home
        assert b.hash() != h0 and b.population() == 5
    with gol.Board(256, 256) as b:
        b.place_rle(oracle.GLIDER, 7, 9)
        h0 = b.hash()
        b.step(4 * 256)
        assert b.hash() == h0


def test_r_pentomino_1103(gol, oracle):
    for k in (1, 16, 32):
        with gol.Board(1024, 1024, gol.BOUNDED, tblock_k=k) as b:
            b.place_rle(oracle.R_PENTOMINO, 511, 511)
            b.step(1103)
            assert b.population() == 116


def test_gosper_gun_long_run_bounded(gol, oracle):
    # bounded 256^2 (Script.fsx:26 board size) gun + R-pentomino, 5000 generations vs the oracle
    b0 = np.zeros((256, 256), np.uint8)
    oracle.place_rle(b0, oracle.GOSPER_GUN, 10, 10)
    oracle.place_rle(b0, oracle.R_PENTOMINO, 180, 150)
    want = oracle.c_run(b0, 5000, 1)
    with gol.Board(256, 256, gol.BOUNDED) as b:
        b.set_cells(b0).step(5000)
        assert np.array_equal(b.get_cells(), want)


# ---------------------------------------------------------------- full-size properties
def _wrapped_region(b, n, x0, y0, ww, wh):
    """Read a window that may wrap around the torus (split into at most 4 in-board regions)."""
    out = np.zeros((wh, ww), np.uint8)
    xs = [(x0, min(ww, n - x0), 0)] + ([(0, ww - (n - x0), n - x0)] if x0 + ww > n else [])
    ys = [(y0, min(wh, n - y0), 0)] + ([(0, wh - (n - y0), n - y0)] if y0 + wh > n else [])
    for (xa, w, ox) in xs:
        for (ya, h, oy) in ys:
            out[oy:oy + h, ox:ox + w] = b.get_region(xa, ya, w, h)
    return out


def test_65536_window_light_cone(gol, oracle):
    """65536^2 torus, splitmix seed, 64 generations: windows of the GPU board equal the oracle run on
    each window grown by the light cone (64 cells per side) -- exact at any board size."""
    n, gens, seed = 65536, 64, 0x5EED
    ww, wh = 160, 96
    with gol.Board(n, n, tblock_k=16) as b:
        b.seed_splitmix(seed)
        b.step(gens)
        for (x0, y0) in ((1000, 2000), (n - 150, 4000), (30000, n - 40), (n - 10, n - 10)):
            xs = (np.arange(x0 - gens, x0 + ww + gens)) % n
            ys = (np.arange(y0 - gens, y0 + wh + gens)) % n
            init = _splitmix_window(seed, n, xs, ys)
            # a bounded run is exact inside the cone: the window's edges never reach the interior
            want = oracle.c_run(init, gens, 1)[gens:gens + wh, gens:gens + ww]
            assert np.array_equal(_wrapped_region(b, n, x0, y0, ww, wh), want), (x0, y0)


def _splitmix_window(seed, width, xs, ys):
    wc = (width + 31) // 32
    chunk = ys[:, None].astype(np.uint64) * np.uint64(wc) + (xs[None, :] // 32).astype(np.uint64)
    import gol_oracle as o

    bits = (o._splitmix64(chunk ^ np.uint64(seed)) & np.uint64(0xFFFFFFFF))
    return ((bits >> (xs[None, :] % 32).astype(np.uint64)) & np.uint64(1)).astype(np.uint8)


def test_65536_temporal_block_invariance(gol):
    """The same 65536^2 run at every layout and depth gives the same board (hash + population)."""
    n = 65536
    res = {}
    with gol.Board(n, n, tblock_k=1, ilv=1) as ref:
        ref.seed_splitmix(7)
        ref.step(48)
        res[(1, 1)] = (ref.hash(), ref.population())
    for ilv, k in ((1, 16), (1, 32), (2, 12), (2, 16), (4, 6), (4, 8)):
        with gol.Board(n, n, tblock_k=k, ilv=ilv) as b:
            b.seed_splitmix(7)
            b.step(48)
            res[(ilv, k)] = (b.hash(), b.population())
    assert len(set(res.values())) == 1, res


# ---------------------------------------------------------------- driver mirror on the GPU
def test_driver_update_view_matches_oracle(gol, oracle):
    from gameoflifewithactors_amd import driver

    frames = []
    agent = driver.UpdateAgent(on_frame=lambda p: frames.append(p.copy()))
    with driver.run(seed=42, agent=agent) as game:
        for _ in range(3):
            game.update_view()
    b = oracle.seed_dotnet(100, 100, 42, 0)
    for i in range(3):
        b = oracle.step(b, 0)
        assert np.array_equal(frames[i], oracle.render_gray8(b, 128))
    fast = driver.UpdateAgent(on_frame=lambda p: frames.append(p.copy()))
    with driver.run(seed=42, agent=fast, emit="pixels") as game:
        game.update_view()
    assert np.array_equal(frames[-1], frames[0])


# ---------------------------------------------------------------- long runs (BASELINE.json configs 2 and 5)
def _golden_long():
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "golden_long.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["c2_4096_torus_dotnet42", "c5_gun_rpent_4096_torus", "c5_gun_rpent_256_bounded"])
@pytest.mark.parametrize("tblock", [0, 1])
def test_long_run_checkpoints(gol, oracle, name, tblock):
    """Every checkpoint (hash + population) of the long-run fixtures -- 4096^2 x 10k generations seeded
    by .NET Random (config 2), Gosper gun + R-pentomino x 100k generations on a 4096^2 torus and the
    256^2 bounded board (config 5) -- at the engine's default temporal block and at k = 1."""
    case = _golden_long()[name]
    with gol.Board(case["width"], case["height"], case["boundary"], tblock_k=tblock) as b:
        if case["init"] == "dotnet-mod2":
            b.seed_dotnet(case["seed"], gol.INIT_DOTNET_MOD2)
        else:
            for pat, x, y in case["patterns"]:
                b.place_rle(getattr(oracle, pat), x, y)
        assert b.hash() == case["initial_hash"]
        done = 0
        for gen, h, pop in case["checkpoints"]:
            b.step(gen - done)
            done = gen
            assert (b.hash(), b.population()) == (h, pop), (name, gen)
        assert b.generation == case["generations"]


@pytest.mark.parametrize("split", [0.95, 0.3, 0.5])
def test_group_split_extremes_match_oracle(gol, oracle, split):
    """Segments shared by the waves of a SIMD (age-ordered shares, plan_stream / group_cut) at extreme
    split fractions -- an empty or near-empty share for some waves -- stay bit-exact (board option "split")."""
    for boundary in (0, 1):
        for w, h, k, ilv in ((4096, 1500, 12, 2), (4096, 700, 16, 2), (2048, 900, 32, 1), (4096, 600, 8, 4)):
            b0 = (np.random.default_rng(w + h + k + boundary).random((h, w)) < 0.4).astype(np.uint8)
            gens = 2 * k + 5
            opts = {"split": int(split * 65536), "coop": 0}
            with gol.Board(w, h, boundary, tblock_k=k, ilv=ilv, options=opts) as b:
                b.set_cells(b0).step(gens)
                np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, gens, boundary),
                                              err_msg=f"{boundary} {w}x{h} k={k} ilv={ilv}")


def test_concurrent_calls_on_one_handle_serialise(gol):
    """The reference's timer may re-enter updateView (GameOfLifeDriver.fs:38-40): concurrent gol_step /
    gol_hash calls on one handle (ctypes drops the GIL) are serialised by the handle's mutex, so the
    result equals the same number of generations run sequentially."""
    import threading

    with gol.Board(1024, 768) as b, gol.Board(1024, 768) as ref:
        b.seed_splitmix(3)
        ref.seed_splitmix(3)
        errors = []

        def worker():
            try:
                for _ in range(10):
                    b.step(5)
                    b.hash()
            except Exception as ex:  # noqa: BLE001
                errors.append(ex)

        threads = [threading.Thread(target=worker) for _ in range(4)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        assert not errors
        ref.step(200)
        assert b.generation == 200 and b.hash() == ref.hash()


def test_native_host_mirror_driver():
    """The C++ host mirror (include/gol/gol_host.hpp): run() / updateView() / the render agent on the
    reference's 100x100 board, frames equal to the oracle's (both emit modes), the timer, the error path
    (tests/cpp/test_host_driver.cpp, built by __graft_entry__.build())."""
    import subprocess

    exe = os.path.join(HERE, "cpp", "build", "test_host_driver")
    assert os.path.exists(exe), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    out = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout + out.stderr
    assert '"failures": []' in out.stdout


# ---------------------------------------------------------------- bounded boards: edge-fill strips
@pytest.mark.parametrize("ilv", [1, 2])
@pytest.mark.parametrize("nblocks", [64, 65, 124, 125, 126, 127, 189, 1024])
def test_bounded_edge_fill_strips_match_oracle(gol, oracle, ilv, nblocks):
    """Bounded boards at least a strip (64 blocks) wide place their first strip at the board's left edge and
    the last at its right edge (the dead cells beyond the edges arrive as the DPP moves' zero fill), and run
    only the trips that produce rows off the board masked (Script.fsx:6-13), in the variant without column
    masks (12-wave workgroups at K = 12).  Every strip-count boundary (nblocks around multiples of 62), the
    top/bottom trips of the first/last segments, a deep block and a remainder pass, against the oracle.  The
    cooperative pass is switched off so the streaming kernel runs every width."""
    w = 32 * ilv * nblocks
    h = 300 if nblocks < 1024 else 64
    b0 = _rand(h, w, nblocks * 10 + ilv, p=0.4)
    for k in (16, 12, 8):
        with gol.Board(w, h, gol.BOUNDED, tblock_k=k, ilv=ilv, options={"coop": 0}) as b:
            assert b.info()["tblock_k"] == k
            b.set_cells(b0).step(2 * k + 5)
            np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 2 * k + 5, 1), err_msg=f"k={k}")


@pytest.mark.parametrize("ilv", [1, 2])
@pytest.mark.parametrize("nblocks", [1, 2, 31, 62, 63])
def test_bounded_narrow_strips_match_oracle(gol, oracle, ilv, nblocks):
    """Bounded boards narrower than one strip (< 64 blocks) take the NARROW streaming variant: lanes off the
    board, column masks at every level (Script.fsx:6-13).  The single-wave, cooperative and LDS-resident
    passes are switched off so the streaming kernel runs, at deep, mid and remainder depths."""
    opts = {"coop": 0, "wave_resident": 0, "resident_max_cells": 0}
    w = 32 * ilv * nblocks
    h = 150
    if w < 3:
        pytest.skip("board narrower than 3 cells")
    b0 = _rand(h, w, nblocks * 7 + ilv, p=0.4)
    for k in (16, 12, 8):
        with gol.Board(w, h, gol.BOUNDED, tblock_k=k, ilv=ilv, options=opts) as b:
            if b.info()["tblock_k"] != k:
                continue  # depth not supported at this layout
            b.set_cells(b0).step(2 * k + 5)
            np.testing.assert_array_equal(b.get_cells(), oracle.c_run(b0, 2 * k + 5, 1), err_msg=f"k={k}")
