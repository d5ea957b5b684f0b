"""Benchmark: cell updates per second (GCUPS) of the hot path on MI355X, plus roofline and CPU baseline.

Workload (BASELINE.json metric "GCUPS at 65536^2 on 1 and 8 x MI355X", config 3 "65536^2 bit-packed
board, 10k generations on one MI355X"): a 65536 x 65536 torus, splitmix random 50 % fill generated on the
device (data: synthetic).  One *step* = one pass of the streaming kernel that advances the whole board by
`tblock` generations (temporal blocking); by default the timed steps cover the whole 10k-generation job.  For N GPUs (one
process per GPU under torchrun) the board is 65536 wide and 65536*N tall, split into N row strips of
65536^2 cells with RCCL halo exchange (weak scaling: per-GPU work fixed).

    python bench.py                          # N = 1: 10k generations timed (~0.5 s), under a minute in all
    python bench.py --steps 64 --warmup 4 --tblock 16
    torchrun --nproc-per-node 8 bench.py --gpus 8

Prints ONE JSON line (rank 0).  Inputs are resident in HBM before the timed region; the timed region is
bracketed by barrier + device synchronize on both sides, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# depths compared by the opt-in on-box autotune (--autotune), per layout (ilv)
AUTOTUNE = {2: [12, 16], 1: [24, 32]}


def default_depth(lib, ilv: int, world: int, boundary: str) -> int:
    """Fixed default temporal depth, so the bench line and a rocprof trace of the same command run the same
    kernel.  Torus, single board or ghost-row strips (N > 1): the engine default K = 12 at M = 2 (12-wave
    workgroups).  Over the whole 10k-generation job it beats K = 16 on both: single board 116.4k vs 109.5k
    GCUPS (profiles/r1/bench_k_ab.log), strips 113.7-114.1k vs 99.2-101.0k (strip_k_ab.log); K = 16 wins only
    on the first passes of a fresh board (ghost_ab2.log).  Bounded boards at M = 2 keep 8-wave workgroups,
    where K = 16 is faster (78.5k vs 74.2k, profiles/r1/strip_bounded_sweep_wpb.log)."""
    if ilv == 2 and boundary == "bounded":
        return 16
    return int(lib.gol_default_tblock(ilv))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md "Chip-level parameters")
# VALU issue peak: 256 CUs x 4 SIMDs, each retiring one full-rate wave64 instruction per 2 cycles (32
# lane-slots per cycle) at 2.4 GHz.
VALU_PEAK_TSLOTS = 256 * 4 * 32 * 2.4e9 / 1e12


def valu_slots_per_word_gen(ilv: int) -> float:
    """Algorithmic VALU issue slots per 32-cell word per generation (gol_bitlogic.h, gol_step.hip): 9
    full-rate v_bitop3_b32 per word, plus per block of `ilv` words 2 v_alignbit_b32 and 2 DPP moves (the
    block-edge words of both neighbour lanes), which are half-rate on gfx950 (2 slots each;
    profiles/r1/valu_rates_gfx950.jsonl)."""
    return 9 + 8 / ilv


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=0,
                   help="timed passes (0 = enough passes for --generations: the whole BASELINE config-3 job)")
    p.add_argument("--generations", type=int, default=10000,
                   help="generations the default run times (BASELINE config 3: 65536^2, 10k generations)")
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--height", type=int, default=65536, help="rows per GPU (board height = height * gpus)")
    p.add_argument("--board", type=int, default=0,
                   help="strong scaling: a fixed board x board torus split over the GPUs (BASELINE config 4: "
                   "262144); overrides --width/--height")
    p.add_argument("--tblock", type=int, default=0,
                   help="generations per pass (0 = the engine's default for the board layout)")
    p.add_argument("--autotune", action="store_true",
                   help="time the AUTOTUNE depths on the box and keep the faster (agreed across ranks)")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--boundary", choices=["torus", "bounded"], default="torus")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU actor baseline sample length")
    p.add_argument("--cpu-board", type=int, default=512, help="CPU actor baseline board side")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="N > 1: nccl (= RCCL over xGMI, the product path) or gloo (host-staged halo; lets "
                   "several ranks share one GPU in rehearsals)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return p.parse_args()


def cpu_baseline(args):
    """The C++ actor-protocol restatement (oracle/actor_protocol.cpp: GameOfLifeLogic.fs:39-71 message for
    message) on this host's cores, bounded sample (~args.cpu_seconds of wall time)."""
    exe = os.path.join(ROOT, "oracle", "build", "actor_protocol")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    threads = max(1, min(16, os.cpu_count() or 1))
    n = args.cpu_board
    out = subprocess.run([exe, str(n), str(n), "0", str(threads), "42", str(args.cpu_seconds), "dotnet-mod2"],
                         check=True, capture_output=True, text=True, timeout=600).stdout
    r = json.loads(out)
    cpu = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": r["cell_updates_per_s"] / 1e9,
        "unit": "GCUPS",
        "cores": threads,
        "kind": "port",
        "sample": f"actor-protocol restatement, {n}x{n} torus, dotnet-mod2 seed 42, {r['generations']} generations "
        f"in {r['seconds']:.1f} s, {r['messages']} messages, {threads} threads on {cpu}",
    }


def load_traffic(path, key):
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(key)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torchrun")
    # one GPU per rank; a gloo rehearsal may place several ranks on one GPU
    dev = local if args.dist_backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    from gameoflifewithactors_amd import TORUS, BOUNDED
    from gameoflifewithactors_amd.strips import StripRunner

    from gameoflifewithactors_amd import _lib

    boundary = TORUS if args.boundary == "torus" else BOUNDED
    if args.board:
        args.width, args.height = args.board, args.board // world  # rows per GPU (last rank may own more)
        W, H = args.board, args.board
    else:
        W, H = args.width, args.height * world
    lib = _lib.load()
    ilv = lib.gol_default_ilv(W)
    # Temporal depth: --tblock, the fixed default, or (--autotune) a short on-box race between the depths
    # that are within a few percent of each other across MI355X boxes.
    if args.tblock:
        cands = [args.tblock]
    elif args.autotune:
        cands = AUTOTUNE.get(ilv, [default_depth(lib, ilv, world, args.boundary)])
    else:
        cands = [default_depth(lib, ilv, world, args.boundary)]
    runner = StripRunner(W, H, boundary, max(cands), rank=rank, world=world, device=torch.device("cuda", dev))
    runner.seed_splitmix(args.seed)
    k, tune = cands[0], None
    if len(cands) > 1:
        per_gen = []
        for kk in cands:
            runner.step_pass(kk)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(runner.compute_stream)
            for _ in range(4):
                runner.step_pass(kk)
            e1.record(runner.compute_stream)
            torch.cuda.synchronize()
            per_gen.append(e0.elapsed_time(e1) / (4 * kk))
        if world > 1:  # every rank must use the same depth (ghost rows, halo messages)
            t = torch.tensor(per_gen, dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            per_gen = [float(x) for x in t]
        k = cands[min(range(len(cands)), key=lambda i: per_gen[i])]
        tune = {str(kk): round(1e3 * pg, 3) for kk, pg in zip(cands, per_gen)}  # us per generation
    runner.k = k
    if args.steps <= 0:  # the whole job: ceil(generations / k) passes of k generations
        args.steps = -(-args.generations // k)

    for _ in range(args.warmup):
        runner.step_pass()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    stream = runner.compute_stream
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        runner.step_pass()
    ev1.record(stream)
    barrier()
    dt = time.perf_counter() - t0
    kernel_s = ev0.elapsed_time(ev1) / 1e3  # HIP events on the stream the step kernels run on
    if world > 1:
        t = torch.tensor([dt, kernel_s], device="cuda" if args.dist_backend == "nccl" else "cpu",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kernel_s = float(t[0]), float(t[1])

    # Memory-side reference point, outside the timed region: the same board streamed by K = 1 passes (the
    # halo-free streaming kernel), HIP events on the compute stream.  Single GPU only.
    k1 = None
    if world == 1 and k > 1:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        runner.step_pass(1)
        e0.record(stream)
        for _ in range(16):
            runner.step_pass(1)
        e1.record(stream)
        torch.cuda.synchronize()
        t1 = e0.elapsed_time(e1) / 1e3 / 16
        k1 = {"bound": "hbm", "achieved": round(2 * W * args.height / 8 / t1 / 1e9, 2), "peak": HBM_PEAK_GBS,
              "unit": "GB/s", "kernel": f"gol_stream_step<K=1, M={ilv}> (halo-free strips)",
              "avg_launch_us": round(t1 * 1e6, 2)}
        k1["frac"] = round(k1["achieved"] / HBM_PEAK_GBS, 4)

    # Measured device-to-device copy rate on this box (torch copy_ of 1 GiB, 512 MiB read + 512 MiB written
    # per copy), outside the timed region: the practical HBM ceiling the roofline fractions sit under.
    copy_gbs = None
    if world == 1:
        a_ = torch.empty(1 << 27, dtype=torch.int32, device="cuda")
        b_ = torch.empty_like(a_)
        b_.copy_(a_)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record()
        for _ in range(10):
            b_.copy_(a_)
        c1.record()
        torch.cuda.synchronize()
        copy_gbs = round(2 * a_.numel() * 4 * 10 / (c0.elapsed_time(c1) / 1e3) / 1e9, 1)
        del a_, b_

    cells = W * H
    gens = args.steps * k
    gcups = cells * gens / dt / 1e9
    # roofline of the dominant kernel, per launch (one launch = one pass of k generations per GPU)
    cells_gpu = W * args.height
    avg_launch_s = runner.kernel_time_per_pass(kernel_s, args.steps)
    alg_bytes = 2 * cells_gpu / 8  # read + write the packed strip once per pass
    achieved_gbs = alg_bytes / avg_launch_s / 1e9
    slots = valu_slots_per_word_gen(ilv)
    valu_tslots = slots * (cells_gpu / 32) * k / avg_launch_s / 1e12
    tr = load_traffic(args.traffic_json, f"{W}x{args.height}_k{k}") or {}
    traffic = tr.get("bytes_per_launch")  # measured HBM bytes per launch (rocprofv3 PMC, calibrated)

    result = None
    if rank == 0:
        result = {
            "metric": "cell updates/sec (GCUPS) at 65536^2 per GPU",
            "value": round(gcups, 3),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.board else "weak",
            "vs_baseline": None,
            "dtype": "u32 (bit-packed cells)",
            "data": "synthetic (splitmix 50% fill generated on device)",
            "config": {
                "workload": f"{W}x{H} {args.boundary} board, {args.steps * k} generations timed in passes of "
                f"{k} (temporal block), {world} row strip(s)",
                "width": W,
                "height": H,
                "generations_per_step": k,
                "generations_timed": args.steps * k,
                "tblock_autotune_us_per_gen": tune,
                "interleave": ilv,
                "boundary": args.boundary,
                "seed": args.seed,
                "parallelism": f"row strips x{world}" + ((" (RCCL halo exchange)" if args.dist_backend == "nccl" else " (gloo host-staged halo)") if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": "profiles/pmc_traffic.json (tools/pmc_traffic.sh)" if traffic else None,
                "kernel": f"gol_stream_step<K={k}, M={ilv}>",
                "alg_bytes_per_launch": alg_bytes,
                "avg_launch_us": round(avg_launch_s * 1e6, 2),
            },
            "roofline_valu": {
                "bound": "valu",
                "achieved": round(valu_tslots, 3),
                "peak": round(VALU_PEAK_TSLOTS, 2),
                "unit": "T lane-slots/s (VALU issue; half-rate ops count 2)",
                "frac": round(valu_tslots / VALU_PEAK_TSLOTS, 4),
                "slots_per_word_gen": slots,
            },
            "effective_hbm_gbs": round(cells * gens / dt * 0.25 / world / 1e9, 1),
            "roofline_k1_stream": k1,
            "hbm_copy_measured_gbs": copy_gbs,
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N = 1 figure (rank 0 only)
            result["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
