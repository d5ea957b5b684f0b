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
    with Board(w, h, tblock_k=8) as b:
        want0 = b.seed_splitmix(seed).hash()
    lb = LocalBoard(w, h, 0, 8, 4)
    lb.seed_splitmix(seed)
    assert lb.hash() == want0  # seeding
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


def _dist_worker(rank, world, port, width, height, boundary, k, gens, seed, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = None
    try:
        from gameoflifewithactors_amd.strips import StripRunner

        torch.cuda.set_device(0)
        r = StripRunner(width, height, boundary, k, rank=rank, world=world, device=torch.device("cuda", 0))
        r.seed_splitmix(seed)
        r.step(gens)
        res = (rank, r.hash(), r.population(), r.generation)
    finally:
        q.put(res if res is not None else (rank, None, None, None))
        dist.destroy_process_group()


@pytest.mark.parametrize("world,boundary,k", [(2, 0, 12), (3, 1, 8)])
def test_multiprocess_strips_match_single_board(world, boundary, k):
    """The bench's N > 1 path -- one process per strip, StripRunner + HipEngine + DistExchange -- with the
    ranks sharing this one GPU over gloo (host-staged halo; RCCL needs one GPU per rank).  Every rank's
    allreduced hash must equal the single-board run."""
    import socket

    import torch.multiprocessing as mp

    from gameoflifewithactors_amd import Board

    width, height, gens, seed = 4096, 600, 50, 31
    with Board(width, height, boundary, tblock_k=k) as b:
        b.seed_splitmix(seed).step(gens)
        want = (b.hash(), b.population())
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, width, height, boundary, k, gens, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    assert all(r[1] is not None for r in res), res
    assert all((r[1], r[2]) == want for r in res), (res, want)
    assert all(r[3] == gens for r in res)


def test_bench_two_ranks_over_gloo():
    """bench.py --gpus 2 end to end (torchrun, two ranks on this GPU, gloo halo): one JSON line."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29613", os.path.join(root, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--height", "4096", "--dist-backend", "gloo", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["value"] > 0 and r["config"]["height"] == 2 * 4096
    assert abs(r["value_per_gpu"] - r["value"] / 2) < 1e-2
    # the one-process C-ABI leg (gol_create_multi, 2 strips on this GPU) ran after the main leg
    h = r["handle_leg"]
    assert h["value"] > 0 and h["strips"] == 2 and len(h["pass_timing_us"]) == 2, h
    assert all(t["edge_done_us"] >= t["edge_wait_us"] >= 0 for t in h["pass_timing_us"])
    _assert_multi_gpu_report(r["multi_gpu"], 2, "gloo")


def _assert_multi_gpu_report(m, world, backend):
    """the N > 1 line's group, devices and the main leg's per-rank halo figures."""
    assert m["backend"] == backend and m["process_group_size"] == world and m["allreduce_rank_count"] == world, m
    assert m["rccl_version"], m  # the RCCL torch links (reported on a gloo rehearsal too)
    assert [x["rank"] for x in m["ranks"]] == list(range(world))
    for x in m["ranks"]:
        assert x["device"] == 0 and x["pci_bus_id"] and x["name"], x  # every rank on this box's one GPU
        t = x["pass_timing_us"]
        assert t["edge_done_us"] >= t["edge_wait_us"] >= 0 and t["interior_us"] > 0, t
    assert m["edge_wait_us_max"] == max(x["pass_timing_us"]["edge_wait_us"] for x in m["ranks"])


def test_bench_two_ranks_strong_scaling_form_over_gloo():
    """The strong-scaling form (--board N: config 4's fixed board split over the ranks) carries the same N > 1
    fields.  A 16384^2 board here, two ranks on this GPU over gloo."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29617", os.path.join(root, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--board", "16384", "--dist-backend", "gloo", "--no-cpu-baseline",
           "--handle-parts", "0", "--no-verify"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["scaling"] == "strong" and r["config"]["width"] == 16384 and r["config"]["height"] == 16384
    _assert_multi_gpu_report(r["multi_gpu"], 2, "gloo")


def test_262144_board_strips_match_single_board():
    """BASELINE.json config 4 geometry: a 262144^2 torus (8 GiB per packed buffer, 2^31 words -- 64-bit
    indexing) as one board and as 8 row strips of 32768 rows (the 8-GPU partition, here in one process),
    same hash and population after 24 generations."""
    from gameoflifewithactors_amd import Board
    from gameoflifewithactors_amd.strips import LocalBoard

    n, gens, seed = 262144, 24, 0xC4
    with Board(n, n, tblock_k=12) as b:
        b.seed_splitmix(seed).step(gens)
        want = (b.hash(), b.population())
    torch.cuda.empty_cache()
    lb = LocalBoard(n, n, 0, 12, 8)
    lb.seed_splitmix(seed)
    lb.step(gens)
    got_hash = lb.hash()
    del lb
    torch.cuda.empty_cache()
    assert got_hash == want[0]


def test_bench_single_gpu_json_contract():
    """bench.py at N = 1: one JSON line with the driver's keys, the roofline object (achieved / peak =
    frac) and the CPU actor baseline (short sample here)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--steps", "4", "--warmup", "1", "--height", "8192",
           "--cpu-seconds", "1", "--cpu-c2", "128"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in r, key
    assert r["n_gpus"] == 1 and r["steps"] == 4 and r["warmup"] == 1 and r["value"] > 0
    assert r["higher_is_better"] is True and r["vs_baseline"] is None and "workload" in r["config"]
    rf = r["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cb = r["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "GCUPS" and cb["value"] > 0 and cb["cores"] >= 1 and cb["sample"]
    assert set(cb["c1_100x100_100gens"]["gcups_by_seed"]) == {"0", "1", "42"} and cb["fair_cpu"]["value"] > 0
    assert r["value_per_gpu"] == r["value"]
