"""GPU tests of the one-process multi-GPU board (gol_create num_gpus > 1 / gol_create_multi, csrc/gol_multi.cpp).

The reference host is one F# process (GameOfLifeDriver.fs:13-41), so the drop-in must be able to spread a
board over several GPUs behind one handle.  Row strips with k ghost rows, peer-copied halo rows, interior
rows overlapping the copies.  The GPU box has one MI355X, so these tests place every strip on device 0
(``devices=[0] * n``): the protocol, the geometry and the stream/event ordering are the ones a node with n
GPUs runs; only the copies stay on one device.  Bar: bit-exact against the oracle and the single board.
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


def _rand(h, w, seed, p=0.5):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


@pytest.mark.parametrize("boundary", [0, 1])
@pytest.mark.parametrize("n", [2, 3, 4])
@pytest.mark.parametrize("tblock", [1, 4, 8, 16])
def test_multi_board_matches_oracle(gol, oracle, boundary, n, tblock):
    w, h, gens = 256, 150, 37  # 37 = passes of several depths plus a remainder
    b0 = _rand(h, w, 1000 * n + tblock + boundary)
    with gol.Board(w, h, boundary, tblock_k=tblock, devices=[0] * n) as b:
        parts = b.parts()
        assert len(parts) == n and sum(p["rows"] for p in parts) == h
        assert [p["y0"] for p in parts] == [h * r // n for r in range(n)]
        b.set_cells(b0).step(gens)
        got = b.get_cells()
        assert b.generation == gens
    np.testing.assert_array_equal(got, oracle.run(b0, gens, boundary))


@pytest.mark.parametrize("ilv", [1, 2, 4])
def test_multi_board_layouts(gol, oracle, ilv):
    w, h, gens = 512, 96, 29
    b0 = _rand(h, w, 77 + ilv)
    with gol.Board(w, h, 0, tblock_k=32, ilv=ilv, devices=[0, 0, 0]) as b:
        b.set_cells(b0).step(gens)
        got = b.get_cells()
    np.testing.assert_array_equal(got, oracle.run(b0, gens, 0))


@pytest.mark.parametrize("boundary", [0, 1])
def test_thin_strips_cap_the_temporal_block(gol, oracle, boundary):
    """8 strips of 5-6 rows: a pass may not reach past one neighbour strip, so the depth is capped by the
    thinnest strip (ghost = k <= rows) and the result is still exact."""
    w, h, gens = 128, 45, 40
    b0 = _rand(h, w, 5 + boundary)
    with gol.Board(w, h, boundary, tblock_k=16, devices=[0] * 8) as b:
        assert max(p["ghost"] for p in b.parts()) <= min(p["rows"] for p in b.parts())
        b.set_cells(b0).step(gens)
        got = b.get_cells()
    np.testing.assert_array_equal(got, oracle.run(b0, gens, boundary))


def test_two_strip_torus_exchanges_with_one_peer_both_ways(gol, oracle):
    """n = 2 on a torus: the up and down neighbour are the same strip."""
    w, h = 64, 32
    b0 = _rand(h, w, 11)
    with gol.Board(w, h, 0, tblock_k=16, devices=[0, 0]) as b:
        b.set_cells(b0).step(100)
        got = b.get_cells()
    np.testing.assert_array_equal(got, oracle.run(b0, 100, 0))


def test_io_across_strips(gol, oracle):
    """Readback, Gray8 render with a stride, regions spanning strips, RLE placed across a strip edge,
    population and hash: all equal to the single board."""
    w, h = 320, 200
    b0 = _rand(h, w, 21, 0.3)
    with gol.Board(w, h, 0, devices=[0] * 3) as m, gol.Board(w, h, 0) as s:
        for b in (m, s):
            b.set_cells(b0).place_rle(oracle.GOSPER_GUN, 100, h // 3 - 5).step(53)
        np.testing.assert_array_equal(m.get_cells(), s.get_cells())
        np.testing.assert_array_equal(m.render_gray8(128, stride=w + 7), s.render_gray8(128, stride=w + 7))
        np.testing.assert_array_equal(m.get_region(17, 40, 250, 130), s.get_region(17, 40, 250, 130))
        np.testing.assert_array_equal(m.get_region(0, 0, w, h), s.get_cells())
        assert (m.population(), m.hash()) == (s.population(), s.hash())
        m.clear()
        assert m.population() == 0 and m.generation == 0


def test_dotnet_seed_and_golden_checkpoints(gol):
    """BASELINE config 2 through the multi-GPU board: 4096^2 torus, .NET Random(42) in the reference's
    creation order, checkpoints of the committed golden fixture up to generation 1000."""
    case = json.load(open(os.path.join(HERE, "golden", "golden_long.json")))["c2_4096_torus_dotnet42"]
    with gol.Board(case["width"], case["height"], case["boundary"], devices=[0] * 4) as b:
        b.seed_dotnet(case["seed"], gol.INIT_DOTNET_MOD2)
        assert b.hash() == case["initial_hash"]
        done = 0
        for gen, hsh, pop in case["checkpoints"]:
            if gen > 1000:
                break
            b.step(gen - done)
            done = gen
            assert (b.hash(), b.population()) == (hsh, pop), gen


@pytest.mark.parametrize("boundary", [0, 1])
def test_full_width_strips_match_single_board(gol, boundary):
    """65536-wide rows (the bench geometry's width, ghost-row kernel variant at the default depth):
    4 strips equal the single board after several passes."""
    w, h, gens = 65536, 2048, 50
    with gol.Board(w, h, boundary, devices=[0] * 4) as m, gol.Board(w, h, boundary) as s:
        for b in (m, s):
            b.seed_splitmix(0x5EED)
        assert m.hash() == s.hash()
        for b in (m, s):
            b.step(gens)
        assert (m.hash(), m.population()) == (s.hash(), s.population())


def test_num_gpus_beyond_visible_devices_is_rejected(gol):
    import torch

    n = torch.cuda.device_count()
    with pytest.raises(ValueError):
        gol.Board(64, 64, num_gpus=n + 1)
    if n >= 2:  # a real multi-GPU node: strips on devices 0..n-1 over xGMI
        with gol.Board(256, 128, 0, num_gpus=n) as b:
            assert [p["device"] for p in b.parts()] == list(range(n))


def test_calls_restore_the_callers_device(gol, oracle):
    """Every C-ABI call switches to the board's device and back (gol_capi.cpp DeviceGuard): a caller whose
    current device is 1 keeps device 1 across create / step / readback / destroy of boards on device 0."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    b0 = _rand(64, 256, 5)
    torch.cuda.set_device(1)
    try:
        for devices in ([0], [0, 0]):
            with gol.Board(256, 64, devices=devices) as b:
                assert torch.cuda.current_device() == 1
                b.set_cells(b0).step(9)
                assert torch.cuda.current_device() == 1
                np.testing.assert_array_equal(b.get_cells(), oracle.run(b0, 9, 0))
                b.hash(), b.population(), b.render_gray8()
                assert torch.cuda.current_device() == 1
            assert torch.cuda.current_device() == 1
        x = torch.zeros(4, device="cuda")
        assert x.device.index == 1
    finally:
        torch.cuda.set_device(0)


def test_transport_on_one_gpu_is_peer_copies(gol):
    """Strips that share a device move their halo rows by peer copies (RCCL needs one rank per GPU); a single
    board has no exchange (gol_transport)."""
    with gol.Board(1024, 256, 0, devices=[0, 0, 0]) as b:
        assert b.transport().startswith("peer:"), b.transport()
    with gol.Board(1024, 256, 0) as b:
        assert b.transport().startswith("none:")


@pytest.mark.parametrize("transport", [1, 2])
@pytest.mark.parametrize("boundary", [0, 1])
def test_distinct_devices_both_transports_match_oracle(gol, oracle, transport, boundary):
    """A node: one strip per GPU, halo rows by peer copies (the default) and by RCCL (transport 2),
    bit-exact against the oracle and reporting the transport it runs.  Skipped on a one-GPU box."""
    n = gol._lib.device_count()
    if n < 2:
        pytest.skip("needs two GPUs")
    w, h, gens = 1024, 40 * n, 45
    b0 = _rand(h, w, 900 + transport + boundary)
    with gol.Board(w, h, boundary, tblock_k=16, devices=list(range(n)), options={"transport": transport}) as b:
        assert b.transport().startswith("rccl:" if transport == 2 else "peer:"), b.transport()
        b.set_cells(b0).step(gens)
        np.testing.assert_array_equal(b.get_cells(), oracle.run(b0, gens, boundary))


@pytest.mark.parametrize("opts", [{"split": -1}, {"seg_rows": 20}, {"seam": -1}])
def test_stream_options_reach_the_strip_launches(gol, oracle, opts):
    """"split", "seg_rows" and "seam" apply to every strip launch of a multi-part board (they were
    silently dropped); results stay exact."""
    w, h, gens = 64 * 140, 300, 29
    b0 = _rand(h, w, 31)
    with gol.Board(w, h, 0, tblock_k=12, ilv=2, devices=[0, 0, 0], options=opts) as b:
        for name, value in opts.items():
            assert b.get_option(name) == value
        b.set_cells(b0).step(gens)
        np.testing.assert_array_equal(b.get_cells(), oracle.run(b0, gens, 0))
