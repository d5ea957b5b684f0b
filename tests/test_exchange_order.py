"""The halo exchange's point-to-point op lists (strips.DistExchange.post, the bench's multi-GPU path) must
pair correctly under NCCL/RCCL semantics, where tags are IGNORED and the sends from rank a to rank b match
b's receives from a in issue order (inside one ncclGroupStart/End).  A slip here would not fail the gloo
tests (gloo matches on tags) but would hang or corrupt the driver's 8-GPU run.

Each rank's op list is captured (no communicator), then every send is delivered to its matching receive
under both policies -- per-peer issue order (NCCL) and (peer, tag) (gloo) -- and every rank's ghost rows
must then hold exactly the global rows the reference topology gives them: torus wrap
(GameOfLifeDriver.fs:21-25), dead outside a bounded board (Script.fsx:6-13).
"""
from collections import defaultdict
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist

from gameoflifewithactors_amd.strips import DistExchange, partition

TORUS, BOUNDED = 0, 1


class _Op:
    def __init__(self, op, tensor, peer, group=None, tag=0):
        self.op, self.tensor, self.peer, self.tag = op, tensor, peer, tag


def _capture(monkeypatch, world, height, boundary, k, width=4):
    """Per rank: (runner stand-in, buffer, captured op list)."""
    captured = {}
    monkeypatch.setattr(dist, "P2POp", _Op)
    ranks = []
    for r in range(world):
        y0, rows = partition(height, world, r)
        g = k
        buf = torch.full((rows + 2 * g, width), -1, dtype=torch.int64)
        buf[g:g + rows] = torch.arange(y0, y0 + rows, dtype=torch.int64)[:, None]  # owned rows carry their id
        up = (r - 1) % world if (boundary == TORUS or r > 0) else None
        down = (r + 1) % world if (boundary == TORUS or r < world - 1) else None
        runner = SimpleNamespace(geom=SimpleNamespace(ghost=g, rows=rows, y0=y0), up=up, down=down)

        def fake_batch(ops, _r=r):
            captured[_r] = list(ops)
            return []

        monkeypatch.setattr(dist, "batch_isend_irecv", fake_batch)
        DistExchange().post(runner, buf, k)
        ranks.append((runner, buf))
    return ranks, captured


def _deliver(ranks, captured, policy):
    sends, recvs = defaultdict(list), defaultdict(list)  # key (src, dst[, tag]) -> ordered ops
    for r, ops in captured.items():
        for o in ops:
            if o.op is dist.isend:
                sends[(r, o.peer) + ((o.tag,) if policy == "gloo" else ())].append(o)
            else:
                assert o.op is dist.irecv
                recvs[(o.peer, r) + ((o.tag,) if policy == "gloo" else ())].append(o)
    assert sorted(sends) == sorted(recvs), "a send has no matching receive (or vice versa): the exchange would hang"
    for key, ss in sends.items():
        rr = recvs[key]
        assert len(ss) == len(rr), key
        for s, d in zip(ss, rr):
            assert s.tensor.shape == d.tensor.shape, key
            d.tensor.copy_(s.tensor)


def _check_ghosts(ranks, height, boundary, k):
    for runner, buf in ranks:
        g, h, y0 = runner.geom.ghost, runner.geom.rows, runner.geom.y0
        for i in range(k):  # top ghost rows: y0 - k .. y0 - 1; bottom: y0 + h .. y0 + h + k - 1
            for row, gy in ((g - k + i, y0 - k + i), (g + h + i, y0 + h + i)):
                if boundary == TORUS:
                    want = gy % height
                else:
                    want = gy if 0 <= gy < height else -1  # never written: the kernel masks these rows dead
                assert int(buf[row, 0]) == want, (y0, row, gy)


@pytest.mark.parametrize("policy", ["nccl", "gloo"])
@pytest.mark.parametrize("world,height,boundary,k", [
    (2, 64, TORUS, 12),    # up == down: two sends and two receives between the same pair of ranks
    (2, 64, BOUNDED, 12),
    (3, 90, TORUS, 12),
    (3, 91, BOUNDED, 8),   # uneven partition
    (4, 100, TORUS, 16),
    (8, 8 * 32, TORUS, 12),
    (8, 8 * 32 + 5, BOUNDED, 12),
])
def test_exchange_ops_pair_under_nccl_and_gloo(monkeypatch, policy, world, height, boundary, k):
    ranks, captured = _capture(monkeypatch, world, height, boundary, k)
    _deliver(ranks, captured, policy)
    _check_ghosts(ranks, height, boundary, k)


def test_world2_torus_order_is_what_makes_nccl_pair_it(monkeypatch):
    """With up == down, NCCL pairs by position only: the op list must interleave as (send top, send bottom,
    recv bottom ghost, recv top ghost) on both ranks.  Swapping the two receives would put each halo in the
    wrong ghost band -- this is caught by the delivery check."""
    ranks, captured = _capture(monkeypatch, 2, 64, TORUS, 4)
    for ops in captured.values():
        assert [o.op for o in ops] == [dist.isend, dist.isend, dist.irecv, dist.irecv]
    swapped = {r: ops[:2] + ops[2:][::-1] for r, ops in captured.items()}
    _deliver(ranks, swapped, "nccl")
    with pytest.raises(AssertionError):
        _check_ghosts(ranks, 64, TORUS, 4)


# ---------------------------------------------------------------- the one-process handle (csrc/gol_multi.cpp)
def _deliver_plan(plan, nparts, height, ghost, boundary, k):
    """Execute gol_exchange_plan's messages under RCCL pairing (per (sender, receiver) in issue order) on buffers
    whose every row holds its global row index (-1 = not written), and check every part's ghost rows."""
    y0 = [height * r // nparts for r in range(nparts)]
    rows = [height * (r + 1) // nparts - y0[r] for r in range(nparts)]
    bufs = []
    for r in range(nparts):
        b = [-1] * (rows[r] + 2 * ghost)
        for i in range(rows[r]):
            b[ghost + i] = y0[r] + i
        bufs.append(b)
    sends, recvs = defaultdict(list), defaultdict(list)
    for part, op, peer, row, n in plan:
        assert n == k
        (sends[(part, peer)] if op == "send" else recvs[(peer, part)]).append((part, row))
    assert sorted(sends) == sorted(recvs), "a send has no matching receive: RCCL would hang"
    for key in sends:
        assert len(sends[key]) == len(recvs[key]), key
        for (sp, srow), (rp, rrow) in zip(sends[key], recvs[key]):
            bufs[rp][rrow:rrow + k] = bufs[sp][srow:srow + k]
    for r in range(nparts):
        for i in range(k):
            for row, gy in ((ghost - k + i, y0[r] - k + i), (ghost + rows[r] + i, y0[r] + rows[r] + i)):
                want = gy % height if boundary == TORUS else (gy if 0 <= gy < height else -1)
                assert bufs[r][row] == want, (r, row, gy)


@pytest.mark.parametrize("nparts,height,boundary,ghost,k", [
    (2, 64, TORUS, 12, 12), (2, 64, TORUS, 12, 8), (2, 64, BOUNDED, 16, 12), (3, 91, TORUS, 8, 8),
    (3, 91, BOUNDED, 8, 4), (4, 100, TORUS, 16, 16), (5, 333, TORUS, 12, 1), (8, 8 * 32, TORUS, 12, 12),
    (8, 8 * 32 + 5, BOUNDED, 12, 12), (8, 65536 * 8, TORUS, 12, 12),
])
def test_handle_exchange_plan_pairs_under_rccl(nparts, height, boundary, ghost, k):
    """The one-process multi-GPU handle (gol_create num_gpus > 1) moves its halo rows with RCCL send/recv when every
    part has its own GPU (csrc/gol_multi.cpp exchange_rccl) and with peer copies otherwise; both execute
    gol_exchange_plan.  Under RCCL pairing (tags ignored, per-peer issue order) every receive must get the rows the
    topology gives it: torus wrap (GameOfLifeDriver.fs:21-25), nothing beyond a bounded board (Script.fsx:6-13)."""
    from gameoflifewithactors_amd import _lib

    plan = _lib.exchange_plan(height, boundary, nparts, ghost, k)
    _deliver_plan(plan, nparts, height, ghost, boundary, k)


def test_handle_exchange_plan_rejects_bad_geometry():
    from gameoflifewithactors_amd import _lib

    with pytest.raises(ValueError):
        _lib.exchange_plan(64, TORUS, 2, 4, 8)  # ghost < k
    with pytest.raises(ValueError):
        _lib.exchange_plan(20, TORUS, 4, 8, 8)  # parts of 5 rows are thinner than k
