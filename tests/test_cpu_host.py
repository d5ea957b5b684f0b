"""CPU tests of the product's host side: the bit logic compiled for the host, the C ABI library's
exports, its no-GPU error behaviour, and the Python mirror of the reference's F# types.
No kernel is launched here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HEADER = os.path.join(ROOT, "include", "gol", "gol.h")


def test_bitlogic_exhaustive_on_host(tmp_path):
    """gol_bitlogic.h (the kernel's 13-op rule) vs GameOfLifeLogic.fs:59-63 on all 3x3 neighbourhoods."""
    exe = tmp_path / "test_bitlogic"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "cpp", "test_bitlogic.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert '"mismatches": 0' in out


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w]+\s*\*?\s*(gol_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    names = _declared_functions()
    for must in ("gol_create", "gol_step", "gol_render_gray8", "gol_hash", "gol_strip_step", "gol_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from gameoflifewithactors_amd import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared_functions():
        assert hasattr(lib, name), f"libgol_hip.so does not export {name}"
        assert name in _lib.SIGNATURES, f"_lib.SIGNATURES lacks a binding for {name}"


def test_debug_option_list_matches_the_library():
    """the test knobs are listed once in the library (csrc/gol_capi.cpp kDebugOptions, exported by
    gol_debug_option_names); the Python routing set _lib.DEBUG_OPTIONS must be exactly that list, or a knob would be
    sent to gol_set_option (GOL_ERR_INVALID) without any test noticing."""
    from gameoflifewithactors_amd import _lib

    names = _lib.load().gol_debug_option_names().decode().split(",")
    assert len(names) == len(set(names))
    assert set(names) == set(_lib.DEBUG_OPTIONS)


def test_layout_choice():
    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    assert [lib.gol_default_ilv(w) for w in (100, 32, 96, 64, 320, 128, 65536)] == [0, 1, 1, 2, 2, 2, 2]
    assert all(lib.gol_supported_k(lib.gol_default_tblock(m), m) for m in (1, 2, 4))
    assert lib.gol_supported_k(32, 1) == 1
    # ilv 4: the streaming pass to K = 8, then K = 16 / 32 on the level-pipelined pass (gol_pipe.hip)
    assert [lib.gol_supported_k(k, 4) for k in (8, 12, 16, 24, 32)] == [1, 0, 1, 0, 1]


@pytest.mark.parametrize("w,h,boundary,want", [
    (65536, 65536, 0, (4, 32)),   # the north-star board: the level-pipelined pass
    (65536, 65536, 1, (4, 32)),   # bounded boards too (round 6: rows of >= 64 blocks)
    (8064, 135000, 1, (2, 12)),   # bounded, 63 blocks: the streaming pass
    (32768, 32768, 0, (4, 32)),   # 2^30 cells
    (65536, 8192, 0, (2, 12)),    # 2^29 cells: below the pass's cut-over (a 65536^2 board as 8 strips)
    (7936, 135400, 0, (4, 32)),   # one full strip of 62 blocks per row
    (7808, 137600, 0, (2, 12)),   # 61 blocks: no full strip
    (65600, 65536, 0, (2, 12)),   # width % 128 != 0
])
def test_default_layout(w, h, boundary, want):
    """gol_default_layout: the layout and depth gol_create picks for a board (or row strip) of this shape."""
    import ctypes

    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    ilv, k = ctypes.c_int(), ctypes.c_int()
    assert lib.gol_default_layout(w, h, boundary, ctypes.byref(ilv), ctypes.byref(k)) == 0
    assert (ilv.value, k.value) == want


@pytest.mark.parametrize("k", [16, 32])
@pytest.mark.parametrize("w,rows,ghost,wrap,wgs", [
    (65536, 65536, 0, 1, 256),    # the bench board: 8 strips + 16 remainder blocks, 3 sub-strips per wave
    (63488, 65536, 0, 1, 256),    # 8 full strips, no remainder
    (8192, 4100, 0, 1, 256),      # 1 strip + 2 blocks: 16 sub-strips per wave
    (16000, 9000, 0, 1, 256),     # 2 strips + 1 block
    (12032, 3000, 0, 1, 256),     # 94 blocks: a remainder of 32 is one more (overlapping) strip
    (65536, 8192, 32, 0, 256),    # an 8-GPU rank's ghost-row strip
    (65536, 65536, 32, 0, 240),   # fewer workgroups (spare waves left for the edge bands)
    (262144, 4096, 0, 1, 256),    # config 4's width (33 strips + 2 blocks), short rows: packing capped by groups
    (65536, 37, 0, 1, 256),       # fewer rows than groups
])
@pytest.mark.parametrize("boundary", [0, 1])
def test_pipe_plan_covers_the_board(k, w, rows, ghost, wrap, wgs, boundary):
    """The level-pipelined pass's plan (gol_pipe.hip plan_pipe), walked on the host (pipe_check_plan): every output
    (row, block) is stored, every row a packed remainder sub-strip reads lies inside the buffer without a wrap or a
    clamp (its rows are sub-strip 0's at a fixed offset), every packed group has the same rows, lane offsets fit 32
    bits, and the grid is one round of `wgs` workgroups where the board allows it."""
    import ctypes

    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    if boundary == 1:  # bounded: rows never wrap; rows of at least 64 blocks
        wrap = 0
        if w < 8192:
            pytest.skip("bounded rows need 64 blocks")
    s = _lib.Strip(w, rows, 0, rows, ghost, w // 32, boundary, wrap, 4, 0)
    plan = (ctypes.c_int64 * 15)()
    assert lib.gol_debug_pipe_plan(ctypes.byref(s), k, 0, rows, wgs, plan, 15) == 0, lib.gol_last_error()
    nstrips, rem, rq, rp, ngroups, grows, pk_lo, pk_hi, npk, nrem, p, split1, split2, grid, bad = plan
    assert bad == 0, list(plan)
    assert p == (4 if k == 16 else 2)
    if nstrips * 1 + (1 if rem else 0) <= wgs and rows >= 64:
        assert grid <= wgs, list(plan)
    if w == 65536 and rows == 65536 and wgs == 256:
        # bounded: 63 + 6 x 62 + 63 blocks in 8 strips, 14 between the last two in remainder sub-strips
        want = (8, 14, 16, 4, 249) if boundary else (8, 16, 18, 3, 252)
        assert (nstrips, rem, rq, rp, grid) == want, list(plan)
    if boundary:  # the two edge strips store 63 blocks each, the others 62, the remainder the rest
        nb = w // 128
        assert nb <= 64 and nstrips == 1 or rem == 0 or 126 + 62 * (nstrips - 2) + rem == nb, list(plan)


def test_library_reports_version_without_gpu():
    from gameoflifewithactors_amd import _lib

    assert b"gfx950" in _lib.load().gol_version()


def test_library_unloads_and_reloads():
    """_lib.unload() dlcloses the library (its device code unregistered before process exit); load()
    maps it again.  In a child process: other tests hold the loaded library."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from gameoflifewithactors_amd import _lib\n"
            "_lib.load(); _lib.unload(); assert _lib._lib is None\n"
            "print(_lib.load().gol_version().decode()); _lib.unload()\n"
            # refused while an object that may call the library is alive, allowed after its release
            "class H: pass\n"
            "h = H(); _lib.load(); _lib.hold(h)\n"
            "try:\n    _lib.unload(); raise SystemExit('unload with a live holder')\n"
            "except _lib.GolError: pass\n"
            "assert _lib._lib is not None\n"
            "_lib.release(h); _lib.unload(); assert _lib._lib is None\n") % root
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "gfx950" in r.stdout


def test_strip_engine_close_lets_the_library_unload():
    """a HipEngine (and a StripRunner that created one) holds the library; close() releases it, so
    _lib.unload() works once the strips are done.  CPU strips (no device memory), in a child process."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import torch\n"
            "from gameoflifewithactors_amd import _lib\n"
            "from gameoflifewithactors_amd.strips import HipEngine, StripRunner\n"
            "e = HipEngine(torch.device('cpu'))\n"
            "try:\n    _lib.unload(); raise SystemExit('unload with a live engine')\n"
            "except _lib.GolError: pass\n"
            "e.close(); e.close(); _lib.unload(); assert _lib._lib is None\n"
            "class Eng(HipEngine):\n"
            "    def alloc(self, geom, stream): return torch.zeros((geom.buffer_rows, geom.pitch), dtype=torch.int32)\n"
            "with Eng(torch.device('cpu')) as own:\n"
            "    r = StripRunner(64, 16, 0, 1, device=torch.device('cpu'), engine=own)\n"
            "    r.close()  # a caller's engine stays held until the caller closes it\n"
            "    assert own in _lib._holders\n"
            "assert own not in _lib._holders\n"
            "_lib.unload(); assert _lib._lib is None\n"
            "print('ok')\n") % root
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert "ok" in r.stdout


def test_arch_check_accepts_only_gfx950():
    """gol_create refuses a board on a non-gfx950 device with GOL_ERR_NO_DEVICE (gol.h): the check's
    decision on the device's gcnArchName, host code, exercised without a GPU."""
    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    for name, ok in ((b"gfx950", 1), (b"gfx950:sramecc+:xnack-", 1), (b"gfx942", 0), (b"gfx942:sramecc+:xnack-", 0),
                     (b"gfx9500", 0), (b"gfx90a", 0), (b"", 0), (None, 0)):
        assert lib.gol_arch_supported(name) == ok, name


def test_hash_finalize_matches_oracle(oracle):
    """gol_hash_finalize is host code: the product's final mix equals the oracle's."""
    from gameoflifewithactors_amd import hash_finalize

    rng = np.random.default_rng(3)
    b = (rng.random((9, 130)) < 0.5).astype(np.uint8)
    # rebuild the oracle's partial sum and finalise it with the product
    h, w = b.shape
    nc = (w + 63) // 64
    padded = np.zeros((h, nc * 64), np.uint8)
    padded[:, :w] = b
    v = np.packbits(padded.reshape(h, nc, 64), axis=2, bitorder="little").view("<u8").reshape(h, nc)
    key = np.arange(h * nc, dtype=np.uint64).reshape(h, nc)
    with np.errstate(over="ignore"):
        acc = int(np.sum(oracle._fmix64(v.astype(np.uint64) ^ oracle._fmix64(key + np.uint64(0x9E3779B97F4A7C15))),
                         dtype=np.uint64))
    assert hash_finalize(acc, w, h) == oracle.board_hash(b)


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure path")
def test_create_fails_loudly_without_gpu():
    from gameoflifewithactors_amd import Board

    with pytest.raises(RuntimeError):
        Board(64, 64)
    with pytest.raises(RuntimeError):  # the multi-GPU board fails the same way (GOL_ERR_NO_DEVICE)
        Board(64, 64, num_gpus=2)
    with pytest.raises(RuntimeError):
        Board(64, 64, devices=[0, 0])


def test_invalid_arguments_rejected_before_device():
    from gameoflifewithactors_amd import Board

    with pytest.raises(ValueError):
        Board(2, 100)  # < 3: the reference's Dictionary never reaches 8 keys (GameOfLifeLogic.fs:58)
    with pytest.raises(ValueError):
        Board(64, 64, boundary=7)
    with pytest.raises(ValueError):
        Board(64, 64, num_gpus=0)
    with pytest.raises(ValueError):
        Board(64, 64, num_gpus=65)
    with pytest.raises(ValueError):
        Board(64, 64, devices=[])
    with pytest.raises(ValueError):
        Board(64, 64, tblock_k=5)


def test_strip_validation_without_gpu():
    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    s = _lib.Strip(width=96, height=10, y0=0, rows=10, ghost=0, pitch=3, boundary=0, wrap_rows=0, ilv=1)
    w, seg = ctypes.c_int64(), ctypes.c_int64()
    assert lib.gol_strip_plan(ctypes.byref(s), 4, 0, 10, ctypes.byref(w), ctypes.byref(seg)) == 0
    assert w.value == 1 and seg.value == 10  # 3 words -> 1 column strip; 10 rows -> 1 segment
    bad = _lib.Strip(width=100, height=10, y0=0, rows=10, ghost=0, pitch=4, boundary=0, wrap_rows=0, ilv=1)
    assert lib.gol_strip_plan(ctypes.byref(bad), 4, 0, 10, None, None) == _lib.GOL_ERR_INVALID
    for ilv, width in ((3, 96), (4, 96), (2, 96)):  # ilv must be 1/2/4 and divide the row into blocks
        bad = _lib.Strip(width=width, height=10, y0=0, rows=10, ghost=0, pitch=3, boundary=0, wrap_rows=0, ilv=ilv)
        assert lib.gol_strip_plan(ctypes.byref(bad), 4, 0, 10, None, None) == _lib.GOL_ERR_INVALID
    # depth 16 exists for ilv 1 and 2 but not 4 (window registers: 5 * ilv * k per lane)
    s4 = _lib.Strip(width=256, height=64, y0=0, rows=64, ghost=0, pitch=8, boundary=0, wrap_rows=0, ilv=4)
    assert lib.gol_strip_plan(ctypes.byref(s4), 16, 0, 64, None, None) == _lib.GOL_ERR_INVALID
    assert lib.gol_strip_plan(ctypes.byref(s4), 8, 0, 64, None, None) == 0
    # a k-generation pass needs k ghost rows when rows do not wrap
    dummy = ctypes.c_void_p(16)
    assert lib.gol_strip_step(ctypes.byref(s), dummy, ctypes.c_void_p(32), 4, 0, 10, None) == _lib.GOL_ERR_INVALID


# ---------------------------------------------------------------- mirror of the F# types
def test_logic_mirror():
    from gameoflifewithactors_amd import logic

    assert logic.grid == logic.Grid(100, 100) and logic.gridProduct == 10000
    order = []
    logic.apply_grid(lambda x, y: order.append((x, y)), logic.Grid(3, 2))
    assert order == [(0, 0), (0, 1), (1, 0), (1, 1), (2, 0), (2, 1)]  # x outer, y inner


def test_update_agent_fills_pixels_like_the_reference():
    from gameoflifewithactors_amd.driver import UpdateAgent
    from gameoflifewithactors_amd.logic import Grid, Location, UpdateView

    frames = []
    agent = UpdateAgent(Grid(3, 2), 128, on_frame=lambda p: frames.append(p.copy()))
    agent.post(UpdateView.Reset())
    for x in range(3):
        for y in range(2):
            agent.post(UpdateView.Update((x + y) % 2 == 0, Location(x, y)))
    assert len(frames) == 1
    assert frames[0].tolist() == [128, 0, 128, 0, 128, 0]  # pixels[x + y*W]


def test_native_host_mirror_fails_loudly_without_gpu():
    """include/gol/gol_host.hpp (the C++ mirror of the reference's F# driver interface): without a GPU,
    creating a board throws gol::Error with GOL_ERR_NO_DEVICE -- no CPU fallback."""
    from gameoflifewithactors_amd import build as b

    exe = b.build_host_tests(verbose=False)
    out = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert '"failures": []' in out.stdout


def _walk_rows(plan, k, rows, ghost, wrap, out_begin, out_end, trip=4):
    """Every buffer row each wave of the seam geometry reads (csrc/gol_step.hip StreamWave + the unit mapping in
    gol_stream_step): sub-strip 0's walk wraps (single board) or clamps (ghost-row strip) for itself, sub-strip j reads
    j * seg rows further; the walk prefetches ceil((len + 2k) / 4) + 1 trips of 4 rows."""
    nstrips, nsegs, seg, seam, rem, rem_p, rem_mid, rem_units = plan
    buf_rows = rows if wrap else rows + 2 * ghost
    packed = (rem_mid + rem_p - 1) // rem_p
    for r in range(rem_units):
        if 1 <= r <= packed:
            sy = 1 + (r - 1) * rem_p
            count = min(1 + rem_mid - sy, rem_p)
        else:
            sy = 0 if r == 0 else r - packed + rem_mid
            count = 1
        b = out_begin + sy * seg
        e = min(b + seg, out_end)
        nsteps = (e - b) + 2 * k
        br = (b - k) % rows if wrap else b - k + ghost
        for _ in range(((nsteps + trip - 1) // trip + 1) * trip):
            row = br if wrap else min(max(br, 0), buf_rows - 1)
            for j in range(count):
                yield r, sy, j, row + j * seg, buf_rows
            br = (0 if br + 1 == rows else br + 1) if wrap else br + 1


@pytest.mark.parametrize("words,ilv,k", [(64, 1, 8), (64, 1, 4), (262, 1, 8), (262, 2, 12), (2052, 2, 12),
                                         (1026, 2, 16), (128, 2, 8), (200, 1, 2)])
def test_seam_remainder_waves_stay_inside_the_buffer(words, ilv, k):
    """Round 4: packed remainder sub-strips of the seam geometry read past the buffer's end (the walk's last,
    unused prefetch trip) -- an illegal-address fault when the next page was unmapped (an 8209 x 40 ragged board).
    The library's own plan (gol_strip_plan_ex, planned here for 4096 resident waves) must keep every row a wave
    reads inside its buffer, on single boards (rows wrap) and ghost-row strips (interior and edge launches)."""
    import ctypes

    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    for rows in list(range(20, 200, 3)) + [300, 1500, 2048, 4099]:
        for wrap in (True, False):
            ghost = 0 if wrap else k
            strip = _lib.Strip(words * 32, rows if wrap else rows * 3, 0 if wrap else rows, rows, ghost,
                               words, 0, 1 if wrap else 0, ilv, 0)
            launches = [(0, rows)] if wrap else [(0, rows), (k, rows - k), (0, k), (rows - k, rows)]
            for b, e in launches:
                if e <= b:
                    continue
                plan = (ctypes.c_int64 * 8)()
                assert lib.gol_strip_plan_ex(ctypes.byref(strip), k, b, e, plan, 8) == 0, lib.gol_last_error()
                plan = list(plan)
                if not plan[3] or not plan[4]:
                    continue
                for r, sy, j, row, buf_rows in _walk_rows(plan, k, rows, ghost, wrap, b, e):
                    assert 0 <= row < buf_rows, (rows, wrap, (b, e), plan, r, sy, j, row)


@pytest.mark.parametrize("wrap,boundary,single,want", [(True, 0, True, (0.66, 0.76)), (False, 1, True, (0.60, 0.72)),
                                                       (False, 0, False, (0.70, 0.0)), (False, 1, False, (0.64, 0.0))])
def test_stream_plan_group_split_defaults(wrap, boundary, single, want):
    """Round 5: the (12, 2) deep pass's three-wave SIMD groups split a segment by two ratios (split, split2), tuned
    per variant at the bench window on SINGLE boards (profiles/r5/split2_confirm_g.jsonl): torus 0.66 /
    0.76, bounded 0.60 / 0.72.  Ghost-row strips (N > 1) were never measured at those values, so they keep round 4's
    single ratio on both boundaries: torus 0.70, bounded 0.64 (split2 0: geometric)."""
    import ctypes

    from gameoflifewithactors_amd import _lib

    lib = _lib.load()
    rows, k, words = 65536, 12, 2048
    ghost = 0 if single else k
    height = rows if single else rows * 2
    strip = _lib.Strip(words * 32, height, 0, rows, ghost, words, boundary, 1 if wrap else 0, 2, 0)
    plan = (ctypes.c_int64 * 10)()
    assert lib.gol_strip_plan_ex(ctypes.byref(strip), k, 0, rows, plan, 10) == 0, lib.gol_last_error()
    assert plan[8] == int(want[0] * 65536) and plan[9] == int(want[1] * 65536), list(plan)
    plan8 = (ctypes.c_int64 * 8)()  # the 8-entry form still works and writes 8 entries
    assert lib.gol_strip_plan_ex(ctypes.byref(strip), k, 0, rows, plan8, 8) == 0
    assert list(plan8) == list(plan)[:8]
