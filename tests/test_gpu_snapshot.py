"""GPU tests of board save/restore (gol_save_packed / gol_load_packed) and RLE export, through the C ABI.

The snapshot layout is the canonical one the hash is defined on, so it is checked bit-exactly against the
oracle's packing (oracle/gol_oracle.py pack64) for every internal layout, the byte board, and the
multi-strip board, and snapshots must move between boards of different layout / GPU count."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


def _canonical(oracle, b):
    h, w = b.shape
    p = np.zeros((h, (w + 63) // 64 * 64), np.uint8)
    p[:, :w] = b
    return oracle.pack64(p)


def _rand(h, w, seed, p=0.4):
    return (np.random.default_rng(seed).random((h, w)) < p).astype(np.uint8)


@pytest.mark.parametrize("w,h,kw", [(256, 70, {"ilv": 1}), (256, 70, {"ilv": 2}), (512, 33, {"ilv": 4}),
                                    (96, 40, {}), (100, 100, {}), (257, 9, {}), (320, 90, {"devices": [0, 0, 0]})])
def test_save_packed_is_canonical(gol, oracle, w, h, kw):
    b0 = _rand(h, w, w + h)
    with gol.Board(w, h, 0, **kw) as b:
        b.set_cells(b0).step(7)
        want = oracle.run(b0, 7, 0)
        np.testing.assert_array_equal(b.save_packed(), _canonical(oracle, want))
        # load the canonical words back (any board of this size), generation restarts at 0
        b.clear().load_packed(_canonical(oracle, b0))
        assert b.generation == 0
        np.testing.assert_array_equal(b.get_cells(), b0)


def test_snapshot_moves_between_layouts_and_gpu_counts(gol, oracle, tmp_path):
    w, h = 1024, 300
    with gol.Board(w, h, 1, devices=[0, 0, 0, 0]) as m:
        m.seed_splitmix(99).step(41)
        path = str(tmp_path / "b.golsnap")
        m.save(path)
        want = m.get_cells()
        h_m = m.hash()
    for kw in ({"ilv": 1}, {"ilv": 4, "tblock_k": 8}, {"devices": [0, 0]}):
        with gol.Board.from_snapshot(path, **kw) as b:
            assert b.boundary == 1 and b.hash() == h_m
            np.testing.assert_array_equal(b.get_cells(), want)
            b.step(13)
            np.testing.assert_array_equal(b.get_cells(), oracle.run(want, 13, 1))


def test_snapshot_hash_is_checked_on_load(gol, tmp_path):
    from gameoflifewithactors_amd import patterns

    with gol.Board(128, 64) as b:
        b.seed_splitmix(5)
        path = str(tmp_path / "b.golsnap")
        b.save(path)
    head, words = patterns.read_snapshot(path)
    words[3] ^= 1
    patterns.write_snapshot(path, words, head["width"], head["height"], head["boundary"], 0, head["hash"])
    with pytest.raises(ValueError):
        gol.Board.from_snapshot(path)


@pytest.mark.parametrize("w,h,kw", [(200, 60, {}), (100, 100, {}), (256, 96, {"devices": [0, 0]})])
def test_rle_export_places_back(gol, oracle, w, h, kw):
    """to_rle (host) -> gol_place_rle (the product's C RLE parser) reproduces the board."""
    with gol.Board(w, h, 0, **kw) as b, gol.Board(w, h, 0, **kw) as c:
        b.place_rle(oracle.GOSPER_GUN, 5, 7).place_rle(oracle.R_PENTOMINO, w // 2, h // 2).step(30)
        c.place_rle(b.to_rle(), 0, 0)
        np.testing.assert_array_equal(c.get_cells(), b.get_cells())


def test_full_size_snapshot_round_trip(gol):
    """65536^2 (BASELINE config 3): 512 MiB canonical snapshot out and back in, hash preserved."""
    with gol.Board(65536, 65536) as b:
        b.seed_splitmix(0x5EED).step(12)
        words = b.save_packed()
        h = b.hash()
    assert words.shape == (65536, 1024)
    with gol.Board(65536, 65536, ilv=1) as c:
        c.load_packed(words)
        assert c.hash() == h
