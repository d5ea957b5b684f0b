"""Every default the boundary header states (include/gol/gol.h, gol_create's tblock_k and num_gpus paragraphs,
gol_transport, gol_set_option "transport") asserted through the C ABI: gol_info / gol_layout / gol_part_info /
gol_transport on single boards of every size class and on a two-part board ("the boundary header
contradicts the code").  Reference seam: GameOfLifeLogic.fs:39 (createCell), GameOfLifeDriver.fs:16-34."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gol():
    import gameoflifewithactors_amd as g
    from gameoflifewithactors_amd import _lib

    _lib.load()
    return g


# (width, height, boundary) -> (packed, ilv, tblock_k), the table in gol.h
CASES = [
    ((100, 100, 0), (False, 0, 8)),          # the reference's own board: byte board, ilv-1 rows below 2^25 cells, k 8
    ((10001, 10001, 0), (False, 0, 16)),     # byte boards below 3 * 2^26 cells: ilv-1 rows, k 16 below 2^27 ...
    ((20001, 10001, 0), (False, 0, 24)),     # ... k 24 above
    ((65535, 8193, 0), (False, 0, 12)),      # from 3 * 2^26 cells: ring rows, the aligned rules (k 12 from 2^29)
    ((30001, 10001, 0), (False, 0, 16)),     # ... k 16 below 2^29 ring cells
    ((10001, 10001, 1), (False, 0, 16)),     # bounded: the same classes (block rows from 3 * 2^26 cells)
    ((20001, 10001, 1), (False, 0, 24)),
    ((30001, 10001, 1), (False, 0, 16)),
    ((65535, 8193, 1), (False, 0, 12)),
    ((1024, 1024, 0), (True, 1, 8)),         # packed below 2^25, not a cooperative-pass width: ilv 1, k 8
    ((4096, 4096, 0), (True, 2, 16)),        # cooperative-pass board 4096 wide: ilv 2, k 16
    ((8192, 8192, 1), (True, 4, 8)),         # cooperative-pass board 8192 wide: ilv 4, k 8
    ((16384, 8192, 0), (True, 2, 16)),       # 2^25 .. 2^29, width % 64 == 0: ilv 2, k 16
    ((32768, 16384, 0), (True, 2, 12)),      # from 2^29: ilv 2, k 12 on the torus ...
    ((32768, 16384, 1), (True, 2, 12)),      # ... and bounded (k 16 until round 3)
    ((32768, 32768, 0), (True, 4, 32)),      # torus from 2^30 cells, width % 128 == 0: the level-pipelined pass
    ((32768, 32768, 1), (True, 4, 32)),      # ... and bounded (rows of >= 64 blocks)
    ((8224, 4096, 0), (True, 1, 32)),        # other packed widths from 2^25 cells: ilv 1, k 32
]


@pytest.mark.parametrize("shape,want", CASES)
def test_single_board_defaults(gol, shape, want):
    w, h, boundary = shape
    with gol.Board(w, h, boundary) as b:
        i = b.info()
        assert (i["packed"], i["ilv"], i["tblock_k"]) == want, i
        assert i["pitch"] == (w // 32 if i["packed"] else 0)
        assert b.parts() == [{"device": b.parts()[0]["device"], "y0": 0, "rows": h, "ghost": 0}]
        assert b.transport().startswith("none:")
        assert b.get_option("transport") == 0
        with pytest.raises(NotImplementedError):  # a single board has no halo exchange
            b.set_option("transport", 2)


def test_two_part_board_defaults(gol):
    """Two strips: balanced rows, ghost = the board's depth capped by the thinnest strip, peer copies by default; RCCL
    refuses two parts on one device and the board keeps peer copies."""
    with gol.Board(4096, 512, 0, devices=[0, 0]) as b:
        i = b.info()
        assert (i["packed"], i["ilv"], i["tblock_k"]) == (True, 1, 8)  # 2^21 cells: ilv 1, k 8 (no cooperative pass)
        assert [(p["y0"], p["rows"], p["ghost"]) for p in b.parts()] == [(0, 256, 8), (256, 256, 8)]
        assert b.transport().startswith("peer:") and b.get_option("transport") == 1
        with pytest.raises(NotImplementedError):
            b.set_option("transport", 2)
        assert b.transport().startswith("peer:")
        with pytest.raises(ValueError):
            b.set_option("transport", 7)
    with gol.Board(4096, 12, 0, tblock_k=16, devices=[0, 0]) as b:  # strips of 6 rows: ghost = 4
        assert [p["ghost"] for p in b.parts()] == [4, 4]
