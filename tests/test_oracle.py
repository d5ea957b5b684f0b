"""CPU tests: pin the oracle (oracle/) before trusting it.

The reference holds no tests or fixtures for this path, so the pins are:
* published .NET Framework System.Random values (the reference's RNG, GameOfLifeDriver.fs:10-11);
* Life known answers (blinker, block, full board, glider period, Gosper gun, R-pentomino);
* agreement of three independent restatements: numpy twin, C stepper, C++ actor protocol
  (GameOfLifeLogic.fs:39-71 message for message, under the Reset->State phase barrier);
* the committed golden fixtures (tests/golden/make_golden.py).
"""
import json
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


# ---------------------------------------------------------------- .NET System.Random
@pytest.mark.parametrize("seed,first", [(0, 1559595546), (1, 534011718), (42, 1434747710)])
def test_dotnet_random_published_values(oracle, seed, first):
    assert oracle.DotNetRandom(seed).next() == first


def test_dotnet_random_python_matches_c(oracle):
    import ctypes

    lib = oracle.c_oracle()
    for seed in (0, 1, 42, -7, 2**31 - 1, -(2**31), 161803398, 123456789):
        buf = ctypes.create_string_buffer(64 * 4 + 16)
        lib.dn_random_init(buf, seed)
        r = oracle.DotNetRandom(seed)
        for i in range(300):
            if i % 3 == 2:
                assert r.next(2) == lib.dn_random_next_max(buf, 2)
            else:
                assert r.next() == lib.dn_random_next(buf)


def test_seed_modes_match_c(oracle):
    for mode in (0, 1):
        for w, h, seed in ((100, 100, 42), (37, 5, -3), (3, 64, 9)):
            assert np.array_equal(oracle.seed_dotnet(w, h, seed, mode), oracle.c_seed_dotnet(w, h, seed, mode))
    assert np.array_equal(oracle.seed_splitmix(200, 17, 0x5EED), oracle.c_seed_splitmix(200, 17, 0x5EED))


def test_seed_dotnet_order_is_x_major(oracle):
    # GameOfLifeDriver.fs:16-19: RNG call k -> cell (x = k / H, y = k % H)
    w, h = 7, 5
    r = oracle.DotNetRandom(11)
    draws = [r.next() % 2 == 0 for _ in range(w * h)]
    b = oracle.seed_dotnet(w, h, 11, 0)
    for k, alive in enumerate(draws):
        assert b[k % h, k // h] == alive


# ---------------------------------------------------------------- stepper agreement
@pytest.mark.parametrize("boundary", [0, 1])
def test_numpy_twin_matches_c_stepper(oracle, boundary):
    rng = np.random.default_rng(1)
    for w, h in ((3, 3), (4, 7), (33, 19), (64, 64), (101, 3)):
        b = (rng.random((h, w)) < 0.4).astype(np.uint8)
        assert np.array_equal(oracle.run(b, 25, boundary), oracle.c_run(b, 25, boundary))


def test_hash_twin_matches_c(oracle):
    rng = np.random.default_rng(2)
    for w, h in ((3, 3), (64, 2), (65, 9), (128, 31), (1000, 3)):
        b = (rng.random((h, w)) < 0.5).astype(np.uint8)
        assert oracle.board_hash(b) == oracle.c_hash(b)


def test_small_boards_rejected(oracle):
    with pytest.raises(ValueError):
        oracle.step(np.zeros((2, 5), np.uint8))


# ---------------------------------------------------------------- known answers (external pins)
def test_blinker_period_two(oracle):
    for bd in (0, 1):
        b = np.zeros((8, 8), np.uint8)
        oracle.place_rle(b, oracle.BLINKER, 2, 3)
        b1 = oracle.step(b, bd)
        assert not np.array_equal(b1, b) and np.array_equal(oracle.step(b1, bd), b)


def test_block_still_life(oracle):
    b = np.zeros((6, 6), np.uint8)
    oracle.place_rle(b, oracle.BLOCK, 2, 2)
    assert np.array_equal(oracle.step(b, 0), b)


def test_full_torus_dies(oracle):
    assert oracle.population(oracle.step(np.ones((8, 8), np.uint8), 0)) == 0


def test_glider_returns_after_4w_on_torus(oracle):
    b = np.zeros((32, 32), np.uint8)
    oracle.place_rle(b, oracle.GLIDER, 5, 9)
    assert np.array_equal(oracle.c_run(b, 128, 0), b)
    assert not np.array_equal(oracle.c_run(b, 64, 0), b)


def test_gosper_gun(oracle):
    b = np.zeros((64, 64), np.uint8)
    oracle.place_rle(b, oracle.GOSPER_GUN, 1, 1)
    assert oracle.population(b) == 36
    assert oracle.population(oracle.run(b, 30, 1)) == 41  # gun + 1 glider


def test_r_pentomino_stabilises_at_116(oracle):
    # 768^2 torus: debris and the six escaping gliders stay clear of the wrap for 1103 generations
    b = np.zeros((768, 768), np.uint8)
    oracle.place_rle(b, oracle.R_PENTOMINO, 383, 383)
    assert oracle.population(oracle.c_run(b, 1103, 0)) == 116


# ---------------------------------------------------------------- actor protocol restatement
def _actor(w, h, gens, threads, seed, init="dotnet-mod2"):
    exe = os.path.join(ROOT, "oracle", "build", "actor_protocol")
    out = subprocess.run([exe, str(w), str(h), str(gens), str(threads), str(seed), "0", init],
                         check=True, capture_output=True, text=True).stdout
    return json.loads(out)


@pytest.mark.parametrize("seed", [0, 1, 42])
def test_actor_protocol_equals_synchronous_oracle_c1(oracle, seed):
    # the reference's default board (100x100 torus), dotnet-mod2 init, 100 generations
    r = _actor(100, 100, 100, 4, seed)
    b = oracle.c_run(oracle.seed_dotnet(100, 100, seed, 0), 100, 0)
    assert r["hash"] == oracle.c_hash(b)
    assert r["population"] == oracle.population(b)
    assert r["messages"] == 100 * (18 * 100 * 100 + 1)  # 18 messages per cell per generation + view reset


def test_actor_protocol_without_barrier_is_schedule_dependent(oracle):
    """without the Reset->State phase barrier the reference protocol is racy.  The
    deterministic racy schedule (racy-seq:S) reproduces it: a fixed schedule seed gives a fixed board,
    different seeds give different boards, and none equals the synchronous step -- which is why parity
    is defined under the barrier."""
    exe = os.path.join(ROOT, "oracle", "build", "actor_protocol")

    def run(schedule):
        out = subprocess.run([exe, "12", "12", "6", "1", "42", "0", "dotnet-mod2", schedule], check=True,
                             capture_output=True, text=True).stdout
        return json.loads(out)

    sync = oracle.c_run(oracle.seed_dotnet(12, 12, 42, 0), 6, 0)
    assert run("barrier")["hash"] == oracle.c_hash(sync)
    racy = [run(f"racy-seq:{s}") for s in (1, 2, 3)]
    assert run("racy-seq:1")["hash"] == racy[0]["hash"]  # reproducible
    assert len({r["hash"] for r in racy}) == 3
    assert all(r["hash"] != oracle.c_hash(sync) for r in racy)
    assert all(r["messages"] == 6 * (18 * 144 + 1) for r in racy)  # same 18 messages per cell per generation


def test_actor_protocol_ragged_board(oracle):
    r = _actor(37, 23, 40, 8, 0x5EED, "splitmix")
    b = oracle.c_run(oracle.seed_splitmix(37, 23, 0x5EED), 40, 0)
    assert r["hash"] == oracle.c_hash(b)


# ---------------------------------------------------------------- golden fixtures
def _golden():
    with open(os.path.join(HERE, "golden", "golden_small.json")) as f:
        return json.load(f)["cases"]


def _initial(oracle, case):
    w, h = case["width"], case["height"]
    if case["init"] == "dotnet-mod2":
        return oracle.seed_dotnet(w, h, case["seed"], 0)
    if case["init"] == "dotnet-next2":
        return oracle.seed_dotnet(w, h, case["seed"], 1)
    if case["init"] == "splitmix":
        return oracle.seed_splitmix(w, h, case["seed"])
    b = np.zeros((h, w), np.uint8)
    pats = {"gosper_gun": oracle.GOSPER_GUN, "r_pentomino": oracle.R_PENTOMINO}
    for name, x, y in case["rle"]:
        oracle.place_rle(b, pats[name], x, y)
    return b


@pytest.mark.parametrize("name", sorted(_golden()))
def test_oracle_reproduces_golden(oracle, name):
    case = _golden()[name]
    bd = 0 if case["boundary"] == "torus" else 1
    b = _initial(oracle, case)
    done = 0
    for cp in sorted(int(c) for c in case["checkpoints"]):
        b = oracle.c_run(b, cp - done, bd)
        done = cp
        want = case["checkpoints"][str(cp)]
        assert str(oracle.c_hash(b)) == want["hash"] and oracle.population(b) == want["population"]


def test_render_gray8_layout(oracle):
    b = np.zeros((3, 4), np.uint8)
    b[1, 2] = 1  # cell (x=2, y=1)
    px = oracle.render_gray8(b, 128, stride=6)
    assert px.shape == (18,) and px[2 + 1 * 6] == 128 and px.sum() == 128


def test_rle_parser(oracle):
    assert sorted(oracle.parse_rle("#C comment\nx = 3, y = 3, rule = B3/S23\nbo$2bo$3o!")) == sorted(
        [(1, 0), (2, 1), (0, 2), (1, 2), (2, 2)]
    )
    assert len(oracle.parse_rle(oracle.GOSPER_GUN)) == 36


# ---------------------------------------------------------------- bit-packed long-run oracle (gol_fast.c)
@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("w,h,threads", [(64, 3, 1), (128, 77, 3), (192, 64, 8), (256, 5, 2)])
def test_fast_oracle_matches_byte_oracle(oracle, boundary, w, h, threads):
    b = (np.random.default_rng(w * h + boundary).random((h, w)) < 0.4).astype(np.uint8)
    got, marks = oracle.fast_run(b, 37, boundary, threads=threads, every=5)
    assert np.array_equal(got, oracle.c_run(b, 37, boundary))
    assert [m[0] for m in marks] == [5, 10, 15, 20, 25, 30, 35]
    mid = oracle.c_run(b, 20, boundary)
    assert marks[3][1:] == (oracle.board_hash(mid), oracle.population(mid))


@pytest.mark.parametrize("boundary", [0, 1])
def test_full_size_generator_matches_byte_oracle(oracle, boundary):
    """oracle/gol_fast_gen (which wrote tests/golden/golden_full.json) on a small board: its packed splitmix
    seeding and every checkpoint equal the byte-per-cell oracle's."""
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "oracle", "build", "gol_fast_gen")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(root, "oracle"), "build/gol_fast_gen"], check=True,
                       stdout=subprocess.DEVNULL)
    w, h, seed = 320, 96, 0x5EED
    out = subprocess.run([exe, str(w), str(h), str(boundary), str(seed), "60", "20", "3"], check=True,
                         capture_output=True, text=True).stdout
    marks = [json.loads(line) for line in out.splitlines()]
    b = oracle.c_seed_splitmix(w, h, seed)
    for m, gen in zip(marks, (0, 20, 40, 60)):
        assert m["generation"] == gen
        assert (m["hash"], m["population"]) == (oracle.board_hash(b), oracle.population(b)), gen
        b = oracle.c_run(b, 20, boundary)


def test_full_size_golden_is_consistent():
    """golden_full.json: every case starts from the splitmix board and has a checkpoint per interval."""
    import json

    with open(os.path.join(os.path.dirname(__file__), "golden", "golden_full.json")) as f:
        full = json.load(f)
    assert {"n1_65536_torus", "n1_65536_bounded", "c4_262144_torus"} <= set(full)
    for c in full.values():
        gens = [m[0] for m in c["checkpoints"]]
        assert gens == list(range(0, c["generations"] + 1, c["every"]))
    # torus and bounded start from the same seeded board
    assert full["n1_65536_torus"]["checkpoints"][0] == full["n1_65536_bounded"]["checkpoints"][0]


def test_fast_oracle_known_answers(oracle):
    b = np.zeros((1024, 1024), np.uint8)
    oracle.place_rle(b, oracle.R_PENTOMINO, 511, 511)
    got, _ = oracle.fast_run(b, 1103, oracle.BOUNDED)
    assert oracle.population(got) == 116
    g = np.zeros((64, 64), np.uint8)
    oracle.place_rle(g, oracle.GLIDER, 3, 7)
    assert np.array_equal(oracle.fast_run(g, 4 * 64)[0], g)


def _golden_long():
    import json

    p = os.path.join(os.path.dirname(__file__), "golden", "golden_long.json")
    with open(p) as f:
        return json.load(f)


@pytest.mark.parametrize("name,gens", [("c2_4096_torus_dotnet42", 100), ("c5_gun_rpent_256_bounded", 2000),
                                       ("c5_gun_rpent_4096_torus", 500)])
def test_long_golden_first_checkpoints_from_byte_oracle(oracle, name, gens):
    """Pin the long-run fixtures' leading checkpoints with the independent byte-per-cell oracle."""
    case = _golden_long()[name]
    if case["init"] == "dotnet-mod2":
        b = oracle.c_seed_dotnet(case["width"], case["height"], case["seed"], 0)
    else:
        b = np.zeros((case["height"], case["width"]), np.uint8)
        for pat, x, y in case["patterns"]:
            oracle.place_rle(b, getattr(oracle, pat), x, y)
    assert oracle.c_hash(b) == case["initial_hash"]
    if case["width"] == 4096 and case["init"] == "patterns":
        # Exact by the light cone: each pattern sits >= gens + 8 cells from the board edges and from the
        # other pattern's cone, so a bounded byte-oracle run on each cone window equals the torus run there
        # and every cell outside both windows stays dead.
        want = np.zeros_like(b)
        for pat, x, y in case["patterns"]:
            x0, y0, x1, y1 = x - gens - 8, y - gens - 8, x + 40 + gens + 8, y + 40 + gens + 8
            assert 0 <= x0 and 0 <= y0 and x1 <= case["width"] and y1 <= case["height"]
            assert not want[y0:y1, x0:x1].any()
            want[y0:y1, x0:x1] = oracle.c_run(b[y0:y1, x0:x1], gens, oracle.BOUNDED)
    else:
        want = oracle.c_run(b, gens, case["boundary"])
    mark = [m for m in case["checkpoints"] if m[0] == gens][0]
    assert (mark[1], mark[2]) == (oracle.board_hash(want), oracle.population(want))
