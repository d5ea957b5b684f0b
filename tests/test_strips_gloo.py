"""CPU tests of the multi-GPU strip protocol (gameoflifewithactors_amd/strips.py) with world_size 2 and 3
over gloo: partitioning, ghost-row halo exchange (DistExchange), boundary handling and the global hash
reduction.  The per-strip compute is the oracle engine (tests/strip_oracle_engine.py); the result must
equal the oracle run on the whole board."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, width, height, boundary, k, gens, seed, q, ilv=1):
    import sys

    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok = False
    try:
        from strip_oracle_engine import OracleEngine

        from gameoflifewithactors_amd.strips import StripRunner

        r = StripRunner(width, height, boundary, k, rank=rank, world=world, device=torch.device("cpu"),
                        engine=OracleEngine(ilv=ilv))
        r.seed_splitmix(seed)
        r.step(gens)
        h = r.hash()
        p = r.population()
        cells = r.get_cells().numpy()
        q.put((rank, h, p, r.geom.y0, cells))
        ok = True
    finally:
        if not ok:
            q.put((rank, None, None, None, None))
        dist.destroy_process_group()


@pytest.mark.parametrize("world,boundary,k,gens,height,ilv", [(2, 0, 4, 13, 40, 1), (2, 1, 4, 13, 40, 1),
                                                              (3, 0, 8, 20, 50, 1), (3, 1, 2, 9, 31, 1),
                                                              (2, 0, 16, 32, 35, 1), (2, 0, 8, 19, 40, 4),
                                                              (3, 1, 4, 11, 33, 2)])
def test_strip_protocol_matches_oracle(oracle, world, boundary, k, gens, height, ilv):
    width, seed = 256, 0x5EED
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, width, height, boundary, k, gens, seed, q, ilv))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    assert all(r[1] is not None for r in res), "a rank failed"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    want = oracle.c_run(oracle.seed_splitmix(width, height, seed), gens, boundary)
    got = np.concatenate([r[4] for r in res], axis=0)
    assert np.array_equal(got, want)
    assert all(r[1] == oracle.board_hash(want) for r in res)  # allreduced hash agrees on every rank
    assert all(r[2] == oracle.population(want) for r in res)


def test_partition_balanced():
    from gameoflifewithactors_amd.strips import partition

    for h in (8, 9, 65536, 100):
        for w in (1, 2, 3, 8):
            parts = [partition(h, w, r) for r in range(w)]
            assert parts[0][0] == 0 and sum(p[1] for p in parts) == h
            for a, b in zip(parts, parts[1:]):
                assert a[0] + a[1] == b[0]
            assert max(p[1] for p in parts) - min(p[1] for p in parts) <= 1
