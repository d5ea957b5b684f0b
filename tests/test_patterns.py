"""CPU tests of the pattern and snapshot formats (gameoflifewithactors_amd/patterns.py), checked against
the oracle's RLE parser (oracle/gol_oracle.py parse_rle / place_rle) and canonical packing (pack64)."""
import numpy as np
import pytest

from gameoflifewithactors_amd import patterns


def _canonical(b):
    """Canonical snapshot rows of any width (pad to a multiple of 64, then the oracle's pack64)."""
    h, w = b.shape
    p = np.zeros((h, (w + 63) // 64 * 64), np.uint8)
    p[:, :w] = b
    import gol_oracle

    return gol_oracle.pack64(p)


@pytest.mark.parametrize("h,w,p", [(1, 1, 1.0), (5, 7, 0.5), (40, 130, 0.3), (64, 64, 0.05), (9, 200, 0.9)])
def test_rle_round_trip_through_the_oracle_parser(oracle, h, w, p):
    b = (np.random.default_rng(h * w).random((h, w)) < p).astype(np.uint8)
    b[0] = 0  # leading empty row
    if h > 3:
        b[h // 2] = 0  # empty row in the middle
    text = patterns.to_rle(b)
    assert text.startswith(f"x = {w}, y = {h}, rule = B3/S23\n") and text.rstrip().endswith("!")
    assert all(len(line) <= 70 for line in text.splitlines()[1:])
    back = oracle.place_rle(np.zeros((h, w), np.uint8), text, 0, 0)
    np.testing.assert_array_equal(back, b)


def test_rle_of_known_patterns(oracle):
    for pat in (oracle.GOSPER_GUN, oracle.R_PENTOMINO, oracle.GLIDER, oracle.BLOCK):
        b = oracle.place_rle(np.zeros((16, 48), np.uint8), pat, 0, 0)
        again = oracle.place_rle(np.zeros((16, 48), np.uint8), patterns.to_rle(b), 0, 0)
        np.testing.assert_array_equal(again, b)
    assert patterns.to_rle(np.zeros((3, 3), np.uint8)).endswith("\n!\n")  # empty board: header + "!"
    assert patterns.to_rle(oracle.place_rle(np.zeros((1, 3), np.uint8), "3o!", 0, 0)).splitlines()[1] == "3o!"


def test_snapshot_file_round_trip(oracle, tmp_path):
    b = (np.random.default_rng(1).random((33, 100)) < 0.4).astype(np.uint8)
    words = _canonical(b)
    path = str(tmp_path / "board.golsnap")
    patterns.write_snapshot(path, words, 100, 33, 1, 1234, oracle.board_hash(b))
    head, back = patterns.read_snapshot(path)
    assert head == {"width": 100, "height": 33, "boundary": 1, "generation": 1234, "hash": oracle.board_hash(b)}
    np.testing.assert_array_equal(back.reshape(words.shape), words)
    np.testing.assert_array_equal(oracle.unpack64(back.reshape(words.shape), 100), b)


def test_snapshot_rejects_bad_files(tmp_path):
    bad = tmp_path / "bad"
    bad.write_bytes(b"NOTASNAP" + bytes(40))
    with pytest.raises(ValueError):
        patterns.read_snapshot(str(bad))
    with pytest.raises(ValueError):
        patterns.write_snapshot(str(tmp_path / "x"), np.zeros(3, np.uint64), 64, 2, 0, 0, 0)
    good = tmp_path / "trunc"
    patterns.write_snapshot(str(good), np.zeros(4, np.uint64), 128, 2, 0, 0, 0)
    good.write_bytes(good.read_bytes()[:-8])
    with pytest.raises(ValueError):
        patterns.read_snapshot(str(good))
