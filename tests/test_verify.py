"""The bench's self-check (gameoflifewithactors_amd/checkpoints.py, bench.py "verify"): CPU tests.

* The golden lookups find the committed checkpoints every bench configuration lands on (BASELINE configs 2-5 and
  the weak-scaling boards of ``bench.py --gpus N``).
* VERDICT round 3, "make every multi-GPU bench line check the board it timed": world-2 torus strips over gloo (the
  bench's StripRunner + DistExchange path, the oracle engine per strip) pass the check, and the same run with the
  two halo receives swapped -- each ghost band filled from the wrong side -- FAILS it.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def test_golden_lookups():
    from gameoflifewithactors_amd import checkpoints as c

    name, case = c.splitmix_case(65536, 65536, 0, 0x5EED)
    assert name == "n1_65536_torus"
    assert c.next_checkpoint(case, 569)[0] == 1000 and c.next_checkpoint(case, 1000)[0] == 1000
    assert c.next_checkpoint(case, 10001) is None
    assert c.splitmix_case(65536, 65536, 1, 0x5EED)[0] == "n1_65536_bounded"
    assert c.splitmix_case(262144, 262144, 0, 0x5EED)[0] == "c4_262144_torus"
    assert c.splitmix_case(65536, 65536, 0, 1)[0] is None
    for n in (2, 4, 8):
        nm, cs = c.splitmix_case(65536, 65536 * n, 0, 0x5EED)
        if nm is None:
            pytest.skip("weak-scaling checkpoints not generated yet (tests/golden/make_golden_full.py w2/w4/w8)")
        assert nm == f"w{n}_65536_torus" and c.next_checkpoint(cs, 569)[0] == 600
    assert c.board_case(4096, 4096, 0, "dotnet-mod2", 42)[0] == "c2_4096_torus_dotnet42"
    assert c.board_case(4096, 4096, 0, "dotnet-mod2", 41)[0] is None
    nm, cs = c.board_case(4096, 4096, 0, "rle:gosper-gun@1000,1000+r-pentomino@3000,3000", 0)
    assert nm == "c5_gun_rpent_4096_torus" and c.initial_mark(cs) == (cs["initial_hash"], cs["initial_population"])
    assert c.board_case(256, 256, 1, "rle:gosper-gun@10,10+r-pentomino@180,150", 0)[0] == "c5_gun_rpent_256_bounded"
    assert c.at_generation(cs, 1000)[0] == 1000 and c.at_generation(cs, 1001) is None


def test_verdict():
    from gameoflifewithactors_amd.checkpoints import verdict

    assert verdict(600, 5, 7, (600, 5, 7), "x")["ok"] is True
    assert verdict(600, 5, 7, (600, 5, 8), "x")["ok"] is False
    assert verdict(600, 5, 7, None, None, {"handle_leg.peer": 5, "handle_leg.rccl": None})["ok"] is True
    assert verdict(600, 5, 7, (600, 5, 7), "x", {"handle_leg.peer": 6})["ok"] is False
    assert verdict(600, 5, 7)["ok"] is None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _SwappedReceives:
    """DistExchange with the two halo receives swapped: the rows from `down` land in the TOP ghost band and the rows
    from `up` in the bottom one (at world 2 on a torus both come from the same rank, so only the data is wrong)."""

    def __init__(self, group=None):
        from gameoflifewithactors_amd.strips import DistExchange

        self.inner = DistExchange(group)

    def post(self, r, buf, k):
        g, h = r.geom.ghost, r.geom.rows
        ops = [dist.P2POp(dist.isend, buf[g:g + k].clone(), r.up, None, tag=1),
               dist.P2POp(dist.isend, buf[g + h - k:g + h].clone(), r.down, None, tag=2)]
        top, bottom = torch.empty_like(buf[g - k:g]), torch.empty_like(buf[g + h:g + h + k])
        ops.append(dist.P2POp(dist.irecv, top, r.down, None, tag=1))     # should land in the bottom ghost band
        ops.append(dist.P2POp(dist.irecv, bottom, r.up, None, tag=2))    # should land in the top ghost band
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        buf[g - k:g].copy_(top)
        buf[g + h:g + h + k].copy_(bottom)
        return []


def _worker(rank, world, port, broken, q):
    import sys

    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = None
    try:
        import gol_oracle as o
        from strip_oracle_engine import OracleEngine

        from gameoflifewithactors_amd import checkpoints
        from gameoflifewithactors_amd.strips import StripRunner

        width, height, k, seed, gens = 256, 48, 4, 0x5EED, 17
        r = StripRunner(width, height, 0, k, rank=rank, world=world, device=torch.device("cpu"),
                        engine=OracleEngine(), exchanger=_SwappedReceives() if broken else None)
        r.seed_splitmix(seed)
        r.step(gens)
        h, p = r.hash(), r.population()
        want = o.c_run(o.seed_splitmix(width, height, seed), gens, 0)
        out = checkpoints.verdict(gens, h, p, (gens, o.board_hash(want), o.population(want)), "oracle")
    finally:
        q.put((rank, out))
        dist.destroy_process_group()


@pytest.mark.parametrize("broken", [False, True])
def test_multi_rank_check_catches_a_mispaired_exchange(broken):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, broken, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v is not None for _, v in res), "a rank failed"
    assert all(v["ok"] is (not broken) for _, v in res), res


def _report_worker(rank, world, port, q):
    import json
    import sys

    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = None
    try:
        from strip_oracle_engine import OracleEngine

        import bench
        from gameoflifewithactors_amd.strips import StripRunner

        r = StripRunner(256, 48, 0, 4, rank=rank, world=world, device=torch.device("cpu"), engine=OracleEngine())
        r.seed_splitmix(0x5EED)
        r.step(8)
        rep = bench.multi_gpu_report(r, None, "gloo", None, probe_passes=2)
        out = json.dumps(rep)  # the line is JSON: the report must serialise as it stands
        assert r.generation == 8 + 2 * 4  # the probe passes advanced the board
    finally:
        q.put((rank, out))
        dist.destroy_process_group()


def test_multi_gpu_report_json_contract():
    """an N > 1 bench line says how many ranks the data-path group connected (all-reduce of
    a 1 per rank), which RCCL, which device and PCI bus each rank ran on, and the main leg's per-rank halo-exchange
    wait and edge-band time (StripRunner.timed_pass).  World 2 over gloo on CPU strips: the fields and their shape."""
    import json

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v is not None for _, v in res), "a rank failed"
    for _, v in res:
        rep = json.loads(v)
        assert rep["backend"] == "gloo"
        assert rep["process_group_size"] == world and rep["allreduce_rank_count"] == world
        assert "rccl_version" in rep and "rccl_library" in rep
        assert [x["rank"] for x in rep["ranks"]] == list(range(world))
        for x in rep["ranks"]:
            assert set(x) >= {"rank", "device", "pci_bus_id", "name", "host", "pass_timing_us", "generations_per_pass"}
            t = x["pass_timing_us"]
            assert t["edge_done_us"] >= t["edge_wait_us"] >= 0 and t["interior_us"] >= 0, t
        assert rep["edge_wait_us_max"] == max(x["pass_timing_us"]["edge_wait_us"] for x in rep["ranks"])
