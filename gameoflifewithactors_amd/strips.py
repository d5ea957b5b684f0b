"""Row-strip decomposition of one board over N GPUs (one process per GPU) with halo exchange.

The reference runs one process with W*H cell actors (GameOfLifeDriver.fs:16-34); its only notion of
"neighbour exchange" is the 8 State / NeighbourState messages per cell (GameOfLifeLogic.fs:47-58).
Here rank r owns the global rows [y0_r, y0_r + rows_r) of a bit-packed board in HBM, plus `k` ghost
rows above and below.  One pass advances k generations:

    1. send my top k owned rows to rank r-1 and my bottom k rows to rank r+1, receive their edge rows
       into my ghost rows (torch.distributed point-to-point: NCCL = RCCL over xGMI on GPUs, gloo on CPU)
    2. meanwhile compute the interior rows [k, rows-k), which need no ghost rows (compute stream)
    3. on a second stream, wait for the exchange only, then compute the boundary rows [0, k) and
       [rows-k, rows): they run as soon as the ghost rows land, in the tail of the interior launch

Torus: ring neighbours (r +- 1) mod N.  Bounded: the end strips have no outer neighbour; rows beyond
the board are dead at every generation (the kernel masks them).  With N = 1 the single strip uses the
wrap-rows layout (no ghosts, one launch per pass).

The compute itself goes through an *engine*; the product engine is `HipEngine` (the C ABI,
gol_strip_* in include/gol/gol.h).  Tests may inject a CPU engine to exercise partitioning and the
exchange protocol with gloo; the product path never falls back to one.

The halo exchange goes through an *exchanger*: `DistExchange` (torch.distributed point-to-point, one
process per GPU -- the bench path) or `LocalExchange` (several strips driven by one process, copied
device-to-device; `LocalBoard` uses it to run N strips on the GPUs of one process).
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import _lib
from ._lib import BOUNDED, TORUS, Strip, check


def partition(height: int, world: int, rank: int) -> tuple[int, int]:
    """Rows owned by `rank`: balanced contiguous strips; returns (y0, rows)."""
    base, extra = divmod(height, world)
    rows = base + (1 if rank < extra else 0)
    y0 = rank * base + min(rank, extra)
    return y0, rows


@dataclass
class Geometry:
    width: int
    height: int
    y0: int
    rows: int
    ghost: int
    pitch: int
    boundary: int
    wrap_rows: bool
    ilv: int = 1  # words per interleaved block (include/gol/gol.h, gol_strip.ilv)

    def strip(self, spare_waves: int = 0) -> Strip:
        return Strip(self.width, self.height, self.y0, self.rows, self.ghost, self.pitch, self.boundary,
                     1 if self.wrap_rows else 0, self.ilv, spare_waves)

    @property
    def buffer_rows(self) -> int:
        return self.rows + 2 * self.ghost


class HipEngine:
    """gol_strip_* through libgol_hip.so on the given CUDA(HIP) device.  No CPU fallback."""

    def __init__(self, device: torch.device):
        self.lib = _lib.load()
        _lib.hold(self)  # _lib.unload() refuses while this engine can still call the library
        self.device = device

    def close(self) -> None:
        """Drop this engine's hold on the library: _lib.unload() -- the documented way to unregister
        the device code before exit under rocprofv3 -- refuses while an engine holds it.  Idempotent;
        the engine must not be used afterwards."""
        _lib.release(self)
        self.lib = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def ilv_for(self, width: int, rows: int | None = None, boundary: int = TORUS) -> int:
        """The engine's layout for a strip of this shape (gol_default_layout: ilv 4 for the level-pipelined pass's
        torus strips); by width alone without `rows` (gol_default_ilv)."""
        if rows is None:
            return int(self.lib.gol_default_ilv(width))
        return self.layout_for(width, rows, boundary)[0]

    def layout_for(self, width: int, rows: int, boundary: int) -> tuple[int, int]:
        """(ilv, k) the engine picks for a strip of `rows` rows (gol_default_layout)."""
        ilv, k = ctypes.c_int(), ctypes.c_int()
        check(self.lib.gol_default_layout(width, rows, boundary, ctypes.byref(ilv), ctypes.byref(k)),
              "gol_default_layout")
        return int(ilv.value), int(k.value)

    def supports_k(self, k: int, ilv: int) -> bool:
        return bool(self.lib.gol_supported_k(k, ilv))

    def largest_k(self, n: int, cap: int, ilv: int) -> int:
        for k in (32, 24, 16, 12, 8, 6, 4, 2, 1):
            if k <= cap and k <= n and self.supports_k(k, ilv):
                return k
        return 1

    def alloc(self, geom: Geometry, stream) -> torch.Tensor:
        """A zeroed strip buffer, allocated and cleared ON `stream` (the strip's compute stream): the
        caching allocator ties a block to the stream it was allocated on, and a fill on the default stream
        would race with the non-blocking compute stream's first kernels."""
        with torch.cuda.stream(stream):
            return torch.zeros((geom.buffer_rows, geom.pitch), dtype=torch.int32, device=self.device)

    def step(self, geom: Geometry, src: torch.Tensor, dst: torch.Tensor, k: int, out_begin: int, out_end: int,
             stream: torch.cuda.Stream, spare_waves: int = 0) -> None:
        s = geom.strip(spare_waves)
        check(self.lib.gol_strip_step(ctypes.byref(s), src.data_ptr(), dst.data_ptr(), k, out_begin, out_end,
                                      stream.cuda_stream), "gol_strip_step")

    def plan_waves(self, geom: Geometry, k: int, out_begin: int, out_end: int) -> int:
        """Waves gol_strip_step launches for these output rows (gol_strip_plan)."""
        waves, seg = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.gol_strip_plan(ctypes.byref(geom.strip()), k, out_begin, out_end, ctypes.byref(waves),
                                      ctypes.byref(seg)), "gol_strip_plan")
        return int(waves.value)

    def seed_splitmix(self, geom: Geometry, buf: torch.Tensor, seed: int, stream) -> None:
        s = geom.strip()
        check(self.lib.gol_strip_seed_splitmix(ctypes.byref(s), buf.data_ptr(), seed & 0xFFFFFFFFFFFFFFFF,
                                               stream.cuda_stream), "gol_strip_seed_splitmix")

    def reduce(self, geom: Geometry, buf: torch.Tensor, what: str, stream) -> torch.Tensor:
        s = geom.strip()
        fn = self.lib.gol_strip_hash_partial if what == "hash" else self.lib.gol_strip_population
        with torch.cuda.stream(stream):  # allocate, clear and accumulate on the strip's stream
            acc = torch.zeros(1, dtype=torch.int64, device=self.device)
            check(fn(ctypes.byref(s), buf.data_ptr(), acc.data_ptr(), stream.cuda_stream), what)
        return acc

    def set_cells(self, geom: Geometry, buf: torch.Tensor, cells_u8: torch.Tensor, stream) -> None:
        s = geom.strip()
        with torch.cuda.stream(stream):
            dev = cells_u8.to(self.device).contiguous()
            check(self.lib.gol_strip_pack(ctypes.byref(s), dev.data_ptr(), buf.data_ptr(), stream.cuda_stream),
                  "gol_strip_pack")
        stream.synchronize()

    def get_cells(self, geom: Geometry, buf: torch.Tensor, stream) -> torch.Tensor:
        s = geom.strip()
        with torch.cuda.stream(stream):
            out = torch.empty((geom.rows, geom.width), dtype=torch.uint8, device=self.device)
            check(self.lib.gol_strip_unpack(ctypes.byref(s), buf.data_ptr(), out.data_ptr(), geom.width, 1,
                                            stream.cuda_stream), "gol_strip_unpack")
            host = out.cpu()
        return host


class StripRunner:
    """One rank's strip of a width x height board; `k` generations per pass."""

    def __init__(self, width: int, height: int, boundary: int, k: int, rank: int = 0, world: int = 1,
                 device: torch.device | None = None, engine=None, group=None, exchanger=None, ilv: int = 0):
        if width % 32:
            raise ValueError("row strips need width % 32 == 0 (bit-packed layout)")
        if boundary not in (TORUS, BOUNDED):
            raise ValueError("bad boundary")
        self.width, self.height, self.boundary, self.k = width, height, boundary, k
        self.rank, self.world, self.group = rank, world, group
        y0, rows = partition(height, world, rank)
        if world > 1 and rows < k:
            raise ValueError(f"strip of {rows} rows is thinner than the temporal block k={k}")
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._own_engine = engine is None  # close() releases an engine this runner created, not a caller's
        self.engine = engine if engine is not None else HipEngine(self.device)
        single = world == 1
        if not ilv:  # the engine's layout for this strip's shape (ilv 4: the level-pipelined pass, k 16 / 32) ...
            ilv_for = getattr(self.engine, "ilv_for", None)
            ilv = ilv_for(width, rows, boundary) if ilv_for else 1
            if ilv_for and not getattr(self.engine, "supports_k", lambda kk, m: True)(k, ilv):
                ilv = ilv_for(width)  # ... unless it does not run the asked depth: the streaming layout by width
        if not getattr(self.engine, "supports_k", lambda kk, m: True)(k, ilv):
            raise ValueError(f"temporal block k={k} is not supported for interleave {ilv}")
        self.geom = Geometry(width, height, y0, rows, 0 if single else k, width // 32, boundary,
                             wrap_rows=single and boundary == TORUS, ilv=ilv)
        self.compute_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else _NullStream()
        # the two k-row edge bands run on their own stream: they wait only for the halo exchange, so they
        # fill the tail of the interior launch instead of queueing behind it
        self.edge_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else _NullStream()
        self.bufs = [self.engine.alloc(self.geom, self.compute_stream), self.engine.alloc(self.geom, self.compute_stream)]
        if self.device.type == "cuda":
            for b in self.bufs:
                b.record_stream(self.edge_stream)  # written by the edge stream too
        self.cur = 0
        self.generation = 0
        self.spare_cap = None  # A/B: at most this many waves held back from the interior launch for the edge bands
        self.up = (rank - 1) % world if (boundary == TORUS or rank > 0) else None
        self.down = (rank + 1) % world if (boundary == TORUS or rank < world - 1) else None
        self.exchanger = exchanger if exchanger is not None else DistExchange(group)

    def close(self) -> None:
        """Wait for this strip's streams, free its buffers and release the engine it created (HipEngine.close), so
        _lib.unload() can run after the strip is done.  Idempotent."""
        if getattr(self, "bufs", None) is None:
            return
        self.compute_stream.synchronize()
        self.edge_stream.synchronize()
        self.bufs = None
        if self._own_engine and hasattr(self.engine, "close"):
            self.engine.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---------------------------------------------------------------- state
    def seed_splitmix(self, seed: int) -> None:
        self.engine.seed_splitmix(self.geom, self.bufs[self.cur], seed, self.compute_stream)
        self.generation = 0

    def set_cells(self, cells_owned) -> None:
        """cells_owned: (rows, width) uint8 of this rank's owned rows."""
        self.engine.set_cells(self.geom, self.bufs[self.cur], torch.as_tensor(cells_owned, dtype=torch.uint8),
                              self.compute_stream)
        self.generation = 0

    def get_cells(self) -> torch.Tensor:
        return self.engine.get_cells(self.geom, self.bufs[self.cur], self.compute_stream)

    # ---------------------------------------------------------------- one pass
    def post_exchange(self, k: int | None = None):
        """Start the halo exchange of the current buffer; returns waitables."""
        k = self.k if k is None else k
        if self.world == 1:
            return []
        with _stream_ctx(self.compute_stream):
            return self.exchanger.post(self, self.bufs[self.cur], k)

    def compute(self, reqs, k: int | None = None, marks: dict | None = None) -> None:
        """Interior rows (overlapping the exchange), wait, then the boundary rows; swap buffers.  `marks` (timed_pass):
        timing marks recorded after the interior launch, at the edge stream's release and after the edge bands."""
        k = self.k if k is None else k
        src, dst = self.bufs[self.cur], self.bufs[self.cur ^ 1]
        h = self.geom.rows
        s = self.compute_stream
        if self.world == 1:
            self.engine.step(self.geom, src, dst, k, 0, h, s)
            _mark(marks, "interior", s)
        else:
            lo, hi = min(k, h), max(h - k, min(k, h))
            e = self.edge_stream
            _wait_stream(e, s)  # previous pass and any host-staged ghost copies are done
            # interior overlaps the exchange; it leaves room on the device for the two edge bands, which
            # then run alongside it as soon as the ghost rows land instead of in its tail
            plan = getattr(self.engine, "plan_waves", None)
            spare = plan(self.geom, k, 0, lo) + plan(self.geom, k, hi, h) if plan else 0
            if self.spare_cap is not None:
                spare = min(spare, self.spare_cap)
            self.engine.step(self.geom, src, dst, k, lo, hi, s, spare_waves=spare)
            _mark(marks, "interior", s)
            with _stream_ctx(e):
                for r in reqs:
                    r.wait()  # the edge stream waits for the received ghost rows
            _mark(marks, "go", e)
            self.engine.step(self.geom, src, dst, k, 0, lo, e)
            self.engine.step(self.geom, src, dst, k, hi, h, e)
            _mark(marks, "edge", e)
            _wait_stream(s, e)  # the pass ends when both streams are done
        self.cur ^= 1
        self.generation += k

    def step_pass(self, k: int | None = None) -> None:
        """Advance k (default self.k) generations: exchange || interior, then boundary rows."""
        self.compute(self.post_exchange(k), k)

    def timed_pass(self, k: int | None = None) -> dict:
        """One pass exactly as step_pass, timed per phase from its start (before the halo exchange is posted): to the
        end of the interior launch, to the edge stream's release (the ghost rows landed: the halo-exchange wait) and
        to the end of the two edge bands (the keys of the handle leg's gol_pass_timing).  HIP events on the streams
        of a GPU strip (synchronised after the pass, not inside it); the host clock on a CPU strip.  bench.py runs a
        few of these after its timed region for the per-rank halo figures of an N > 1 line."""
        marks: dict = {}
        _mark(marks, "start", self.compute_stream)
        self.compute(self.post_exchange(k), k, marks)
        start = marks.pop("start")
        if isinstance(start, float):
            us = {n: (t - start) * 1e6 for n, t in marks.items()}
        else:
            torch.cuda.synchronize(self.device)
            us = {n: start.elapsed_time(ev) * 1e3 for n, ev in marks.items()}
        out = {"interior_us": round(us["interior"], 2)}
        if "go" in us:
            out["edge_wait_us"] = round(us["go"], 2)
            out["edge_done_us"] = round(us["edge"], 2)
        return out

    def step(self, generations: int) -> None:
        while generations > 0:
            k = self.k if generations >= self.k else self._largest_k(generations)
            self.step_pass(k)
            generations -= k

    def _largest_k(self, n: int) -> int:
        fn = getattr(self.engine, "largest_k", None)
        return fn(n, self.k, self.geom.ilv) if fn else _largest_k(n)

    def launches_per_pass(self) -> int:
        return 1 if self.world == 1 else 3

    def kernel_time_per_pass(self, total_s: float, passes: int) -> float:
        return total_s / passes

    # ---------------------------------------------------------------- observables (global)
    def _reduce(self, what: str) -> int:
        acc = self.engine.reduce(self.geom, self.bufs[self.cur], what, self.compute_stream)
        if self.device.type == "cuda":
            self.compute_stream.synchronize()
        if self.world > 1:
            if acc.is_cuda and dist.get_backend(self.group) == "gloo":
                acc = acc.cpu()  # gloo reduces host tensors
            dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=self.group)
        return int(acc.item()) & 0xFFFFFFFFFFFFFFFF

    def population(self) -> int:
        return self._reduce("population")

    def hash(self) -> int:
        return int(_lib.load().gol_hash_finalize(self._reduce("hash"), self.width, self.height))


class DistExchange:
    """Halo exchange with torch.distributed point-to-point ops (NCCL = RCCL over xGMI on GPUs, gloo on
    CPU).  Every rank issues its ops in the same order, so NCCL's in-order matching per peer pairs
    them even when up == down (two ranks on a torus); gloo matches on the tags."""

    def __init__(self, group=None):
        self.group = group

    def post(self, r: "StripRunner", buf: torch.Tensor, k: int):
        if buf.is_cuda and dist.get_backend(self.group) == "gloo":
            return self._post_staged(r, buf, k)
        g, h = r.geom.ghost, r.geom.rows
        ops = []
        if r.up is not None:  # my top rows -> up's bottom ghost
            ops.append(dist.P2POp(dist.isend, buf[g:g + k], r.up, self.group, tag=1))
        if r.down is not None:  # my bottom rows -> down's top ghost
            ops.append(dist.P2POp(dist.isend, buf[g + h - k:g + h], r.down, self.group, tag=2))
        if r.down is not None:
            ops.append(dist.P2POp(dist.irecv, buf[g + h:g + h + k], r.down, self.group, tag=1))
        if r.up is not None:
            ops.append(dist.P2POp(dist.irecv, buf[g - k:g], r.up, self.group, tag=2))
        return dist.batch_isend_irecv(ops) if ops else []

    def _post_staged(self, r: "StripRunner", buf: torch.Tensor, k: int):
        """gloo moves host tensors only: stage the edge rows through host memory, synchronously (no
        overlap).  Lets the GPU strip path run over gloo, e.g. several ranks sharing one GPU in tests;
        the multi-GPU bench uses NCCL (RCCL), which sends device memory directly."""
        g, h = r.geom.ghost, r.geom.rows
        ops, recvs = [], []
        if r.up is not None:
            ops.append(dist.P2POp(dist.isend, buf[g:g + k].cpu(), r.up, self.group, tag=1))
        if r.down is not None:
            ops.append(dist.P2POp(dist.isend, buf[g + h - k:g + h].cpu(), r.down, self.group, tag=2))
        if r.down is not None:
            t = torch.empty((k, buf.shape[1]), dtype=buf.dtype)
            ops.append(dist.P2POp(dist.irecv, t, r.down, self.group, tag=1))
            recvs.append((g + h, t))
        if r.up is not None:
            t = torch.empty((k, buf.shape[1]), dtype=buf.dtype)
            ops.append(dist.P2POp(dist.irecv, t, r.up, self.group, tag=2))
            recvs.append((g - k, t))
        for w in dist.batch_isend_irecv(ops) if ops else []:
            w.wait()
        for row, t in recvs:
            buf[row:row + k].copy_(t)
        return []


class LocalExchange:
    """Halo exchange between strips driven by ONE process (device-to-device copies, peer copies across
    GPUs).  All strips must post before any computes (LocalBoard does this)."""

    def __init__(self):
        self.runners: list[StripRunner] = []

    def post(self, r: "StripRunner", buf: torch.Tensor, k: int):
        g, h = r.geom.ghost, r.geom.rows
        if r.up is not None:
            u = self.runners[r.up]
            ub = u.bufs[u.cur]
            buf[g - k:g].copy_(ub[u.geom.ghost + u.geom.rows - k:u.geom.ghost + u.geom.rows], non_blocking=True)
        if r.down is not None:
            d = self.runners[r.down]
            db = d.bufs[d.cur]
            buf[g + h:g + h + k].copy_(db[d.geom.ghost:d.geom.ghost + k], non_blocking=True)
        return []


class LocalBoard:
    """N row strips of one board driven by one process (strip i on devices[i % len(devices)]).
    Used to exercise the strip kernels and ghost geometry on a single GPU, and as an in-process
    multi-GPU mode."""

    def __init__(self, width: int, height: int, boundary: int, k: int, nstrips: int, devices=None, engine_factory=None,
                 ilv: int = 0):
        devices = devices or [torch.device("cuda", torch.cuda.current_device())]
        self.exchange = LocalExchange()
        self.runners = []
        for i in range(nstrips):
            dev = devices[i % len(devices)]
            eng = engine_factory(dev) if engine_factory else None
            r = StripRunner(width, height, boundary, k, rank=i, world=nstrips, device=dev, engine=eng,
                            exchanger=self.exchange, ilv=ilv)
            self.runners.append(r)
        self.exchange.runners = self.runners
        self.width, self.height, self.k = width, height, k

    def _sync_all(self):
        for r in self.runners:
            r.compute_stream.synchronize()

    def close(self) -> None:
        for r in self.runners:
            r.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def step_pass(self, k: int | None = None) -> None:
        self._sync_all()  # every strip's current buffer is final before anyone copies from it
        reqs = [r.post_exchange(k) for r in self.runners]
        self._sync_all()  # ghost rows landed before anyone overwrites a neighbour's source buffer
        for r, q in zip(self.runners, reqs):
            r.compute(q, k)

    def step(self, generations: int) -> None:
        while generations > 0:
            k = self.k if generations >= self.k else self.runners[0]._largest_k(generations)
            self.step_pass(k)
            generations -= k

    def set_cells(self, cells) -> None:
        for r in self.runners:
            r.set_cells(cells[r.geom.y0:r.geom.y0 + r.geom.rows])

    def get_cells(self):
        self._sync_all()
        return torch.cat([r.get_cells() for r in self.runners], dim=0)

    def seed_splitmix(self, seed: int) -> None:
        for r in self.runners:
            r.seed_splitmix(seed)

    def _sum(self, what: str) -> int:
        total = 0
        for r in self.runners:
            acc = r.engine.reduce(r.geom, r.bufs[r.cur], what, r.compute_stream)
            r.compute_stream.synchronize()
            total = (total + int(acc.item())) & 0xFFFFFFFFFFFFFFFF
        return total

    def hash(self) -> int:
        return int(_lib.load().gol_hash_finalize(self._sum("hash"), self.width, self.height))

    def population(self) -> int:
        return self._sum("population")


def _largest_k(n: int) -> int:
    for k in (32, 24, 16, 8, 4, 2, 1):
        if k <= n:
            return k
    return 1


class _NullStream:
    cuda_stream = 0

    def synchronize(self):
        pass


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _mark(marks, name: str, stream) -> None:
    """A timing mark of timed_pass: a timing event recorded on `stream` (GPU strip), else the host clock."""
    if marks is None:
        return
    if isinstance(stream, torch.cuda.Stream):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        marks[name] = ev
    else:
        marks[name] = time.perf_counter()


def _wait_stream(waiter, other) -> None:
    if isinstance(waiter, torch.cuda.Stream):
        waiter.wait_stream(other)


def _stream_ctx(s):
    return torch.cuda.stream(s) if isinstance(s, torch.cuda.Stream) else _NullCtx()
