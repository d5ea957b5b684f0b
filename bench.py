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
    # BASELINE configs 2 and 5 on the C-ABI board (the product's pass choice), one gol_step call per step:
    python bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --steps 5
    python bench.py --init rle:gosper-gun@1000,1000+r-pentomino@3000,3000 --width 4096 --height 4096 \
        --generations 100000 --steps 1 --warmup 1

Prints ONE JSON line (rank 0).  Inputs are resident in HBM before the timed region; the timed region is
bracketed by barrier + device synchronize on both sides, max over ranks.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# depths raced on the box before the timed region (default; --no-autotune skips it), per layout (ilv); ilv 4 (the
# level-pipelined pass) runs its one default depth
AUTOTUNE = {2: [12, 16], 1: [24, 32]}


def default_layout(lib, width: int, rows: int, boundary: int) -> tuple[int, int]:
    """The engine's (ilv, K) for a strip of `rows` rows (gol_default_layout), fixed so the bench line and a rocprof
    trace of the same command run the same kernel.  Torus strips of >= 2^30 cells (the 65536^2 board per GPU): ilv 4
    and K = 32 on the level-pipelined pass (gol_pipe.hip).  Otherwise the streaming pass's K = 12 at
    M = 2 (12-wave workgroups): over the whole 10k-generation job it beat K = 16 on the single board (116.4k vs 109.5k
    GCUPS, profiles/r1/bench_k_ab.log) and on strips (113.7-114.1k vs 99.2-101.0k, strip_k_ab.log); bounded boards
    too since round 3's staged passes (127.5k vs 119.2k GCUPS, profiles/r3/bench_bounded_job_d.log)."""
    import ctypes

    ilv, k = ctypes.c_int(), ctypes.c_int()
    if lib.gol_default_layout(width, rows, boundary, ctypes.byref(ilv), ctypes.byref(k)) != 0:
        raise SystemExit(f"gol_default_layout: {lib.gol_last_error().decode()}")
    return int(ilv.value), int(k.value)


def kernel_name(ilv: int, k: int) -> str:
    """The dominant kernel of a pass of depth k at layout ilv (the name rocprofv3 reports, template arguments
    aside)."""
    if ilv == 4 and k in (16, 32):
        return f"gol_pipe_step<D=4, S={k // 4}, P={64 // k}> (K={k}, M=4)"
    return f"gol_stream_step<K={k}, M={ilv}>"

def hot_kernel_symbol(ilv: int, k: int) -> str:
    """The kernel whose code object keys this configuration's PMC measurements (_lib.device_code_fingerprint): the
    level-pipelined pass (csrc/gol_pipe.hip) at ilv 4 and K = 16 / 32, the streaming pass (csrc/gol_step.hip)
    otherwise."""
    return "gol_pipe_step" if ilv == 4 and k in (16, 32) else "gol_stream_step"


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


def _rccl_version():
    """RCCL's version as the torch build links it ("2.27.7"), or None (no RCCL in this torch)."""
    try:
        import torch

        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 -- a report field, not a failure
        return None


def _mapped_rccl():
    """The librccl this process has mapped (/proc/self/maps), or None: which RCCL actually served the group."""
    try:
        with open("/proc/self/maps") as f:
            libs = sorted({line.split()[-1] for line in f if "librccl" in line and "/" in line})
        return libs or None
    except OSError:
        return None


def _device_identity(dev) -> dict:
    """{device, pci_bus_id, name} of this rank's GPU (hipDeviceProp_t through torch), or nulls on a CPU strip."""
    import torch

    if dev is None or not torch.cuda.is_available():
        return {"device": None, "pci_bus_id": None, "name": None}
    p = torch.cuda.get_device_properties(dev)
    bus = getattr(p, "pci_bus_id", None)
    pci = None
    if bus is not None:
        pci = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), bus, getattr(p, "pci_device_id", 0))
    return {"device": int(dev), "pci_bus_id": pci, "name": p.name}


def multi_gpu_report(runner, dev, backend: str, host_group=None, probe_passes: int = 4) -> dict:
    """What an N > 1 line needs to answer "did RCCL see N ranks, on which GPUs, and what did the halo cost?"
    (VERDICT round 5, item 4).  Collective: every rank calls it, after the timed region; rank 0 gets the full dict.

    * `process_group_size`: torch.distributed's world size; `allreduce_rank_count`: the sum of a 1 from every rank
      all-reduced over the data-path group (RCCL when the backend is nccl) -- N only if RCCL connected all N ranks.
    * `rccl_version` / `rccl_library`: the RCCL torch links and the librccl mapped into this process.
    * `ranks`: per rank (all-gathered over the host group) its device, PCI bus id, device name, host, and the main
      leg's per-phase pass timing: `probe_passes` passes exactly as timed (StripRunner.timed_pass, HIP events):
      interior launch end, halo-exchange wait (edge stream released) and edge-band end, from the pass start, in us.
    * `edge_wait_us_max`: the slowest rank's mean halo wait.
    The probe passes advance the board (the self-check steps on from wherever it is)."""
    import torch
    import torch.distributed as dist

    probes = [runner.timed_pass() for _ in range(probe_passes)]
    timing = {key: round(sum(p[key] for p in probes) / len(probes), 2) for key in probes[0]} if probes else {}
    cuda = backend == "nccl"
    one = torch.ones(1, dtype=torch.int64, device=torch.device("cuda", dev) if cuda else "cpu")
    dist.all_reduce(one)  # over the default (data-path) group: RCCL for nccl
    me = {"rank": dist.get_rank(), **_device_identity(dev if (dev is not None and torch.cuda.is_available()) else None),
          "host": platform.node(), "pass_timing_us": timing, "generations_per_pass": runner.k}
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me, group=host_group)
    waits = [r["pass_timing_us"].get("edge_wait_us") for r in ranks if r and r["pass_timing_us"]]
    return {
        "backend": backend,
        "rccl_version": _rccl_version() if cuda or torch.cuda.is_available() else None,
        "rccl_library": _mapped_rccl(),
        "process_group_size": dist.get_world_size(),
        "allreduce_rank_count": int(one.item()),
        "ranks": ranks,
        "edge_wait_us_max": max(waits) if waits and None not in waits else None,
        "probe_passes": probe_passes,
        "timing": "StripRunner.timed_pass: HIP events on the strip's compute and edge streams, from the pass start "
                  "(before the halo exchange is posted); means over the probe passes, run after the timed region",
    }


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
    p.add_argument("--ilv", type=int, default=0, choices=(0, 1, 2, 4),
                   help="main leg: words per interleaved block (0 = the engine's choice for the strip, gol_default_layout; "
                   "2 with --tblock 12 = the round-5 streaming pass at 65536^2)")
    p.add_argument("--no-autotune", action="store_true",
                   help="skip the on-box race between the AUTOTUNE depths (default: race them during warmup, "
                   "interleaved, and time the faster; agreed across ranks) and use the engine default depth")
    p.add_argument("--seed", type=int, default=0x5EED)
    p.add_argument("--init", default="splitmix",
                   help="board init: splitmix (device-side, the default), dotnet-mod2 (GameOfLifeDriver.fs:9-19), "
                   "dotnet-next2 (Script.fsx:25-27), or rle:SPEC[+SPEC] with SPEC = FILE|gosper-gun|r-pentomino[@x,y]; "
                   "anything but splitmix times the C-ABI board (gol_step: the pass the product picks for the size)")
    p.add_argument("--gens-per-step", type=int, default=0,
                   help="board leg (--init other than splitmix): generations per gol_step call (0 = --generations)")
    p.add_argument("--boundary", choices=["torus", "bounded"], default="torus")
    p.add_argument("--cpu-seconds", type=float, default=8.0,
                   help="CPU baseline sample length (C2 actor sample, fair-CPU sample)")
    p.add_argument("--cpu-c2", type=int, default=4096,
                   help="board side of the C2 actor sample (BASELINE config 2: 4096; smaller for quick checks)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="N > 1: nccl (= RCCL over xGMI, the product path) or gloo (host-staged halo; lets "
                   "several ranks share one GPU in rehearsals)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--handle-leg-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--handle-timeout", type=float, default=300.0,
                   help="seconds the one-process handle leg (a child process of rank 0) may take")
    p.add_argument("--handle-parts", type=int, default=-1,
                   help="one-process C-ABI leg (gol_create / gol_create_multi, csrc/gol_multi.cpp: what the F# "
                   "drop-in calls, run without torch on the library's own HIP runtime): the same board in P row "
                   "strips on devices 0..P-1 (round-robin over the visible devices, so a one-GPU box rehearses it "
                   "with every strip on device 0), timed by rank 0 after the main leg and hashed at the main leg's "
                   "verify generation; -1 = the world size (1: the single board); 0 = off")
    p.add_argument("--verify-gen", type=int, default=-1, help=argparse.SUPPRESS)
    p.add_argument("--handle-first-gen", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--handle-transport", choices=["default", "rccl"], default="default", help=argparse.SUPPRESS)
    p.add_argument("--no-verify", action="store_true",
                   help="skip the untimed self-check (step to the next golden checkpoint and compare hashes)")
    return p.parse_args()


def _cpu_model() -> str:
    cpu = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def _run_json(cmd, timeout=900):
    return json.loads(subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout).stdout)


def cpu_baseline(args):
    """CPU baselines on this host's cores, outside the timed region, rank 0 at N = 1.

    The reference's actors, restated message for message (oracle/actor_protocol.cpp: GameOfLifeLogic.fs:39-71
    under the Reset->State barrier, 18 messages per cell per generation, the driver of
    GameOfLifeDriver.fs:13-41), timed at
      * C1: the reference's own board, 100^2 torus, dotnet-mod2 seeds 0 / 1 / 42, 100 generations each;
      * C2: 4096^2 torus, dotnet-mod2 seed 42, a bounded sample of whole generations (>= 1; ~14 GB of actor
        state -- the largest board timed: 65536^2 as actors would need ~3.6 TB).
    `value` is the C2 figure.  `fair_cpu`: the bit-sliced multithreaded stepper (oracle/gol_fast.c, the
    carry-save oracle) on the bench workload itself, 65536^2 torus, a bounded sample."""
    odir = os.path.join(ROOT, "oracle", "build")
    exe, fast = os.path.join(odir, "actor_protocol"), os.path.join(odir, "gol_fast_bench")
    if not (os.path.exists(exe) and os.path.exists(fast)):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    # the box's CPU share is 16 threads per GPU (OMP_NUM_THREADS there); the host itself has more cores
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, min(16, avail))
    cpu = _cpu_model()
    c1 = {}
    for seed in (0, 1, 42):
        r = _run_json([exe, "100", "100", "100", str(threads), str(seed), "0", "dotnet-mod2"])
        c1[str(seed)] = {"gcups": r["cell_updates_per_s"] / 1e9, "seconds": round(r["seconds"], 3),
                         "generations": r["generations"], "messages": r["messages"], "hash": str(r["hash"])}
    n2 = str(args.cpu_c2)
    c2 = _run_json([exe, n2, n2, "0", str(threads), "42", str(args.cpu_seconds), "dotnet-mod2"])
    fair = _run_json([fast, str(args.width), str(args.width), "0", str(threads), str(args.cpu_seconds)])
    # the same stepper on every CPU this process may run on (the whole host unless the box restricts it)
    fair_all = None
    if avail > threads:
        fair_all = _run_json([fast, str(args.width), str(args.width), "0", str(avail), str(args.cpu_seconds)])
    host = {"logical_cpus": os.cpu_count(), "cpus_available": avail, "model": cpu}
    return {
        "value": c2["cell_updates_per_s"] / 1e9,
        "unit": "GCUPS",
        "cores": threads,
        "kind": "port",
        "sample": f"actor-protocol restatement (oracle/actor_protocol.cpp), C2 {n2}x{n2} torus, dotnet-mod2 seed "
        f"42, {c2['generations']} generation(s) in {c2['seconds']:.1f} s, {c2['messages']} messages, {threads} "
        f"threads on {cpu}",
        "c1_100x100_100gens": {
            "gcups_by_seed": {k: round(v["gcups"], 6) for k, v in c1.items()},
            "seconds_by_seed": {k: v["seconds"] for k, v in c1.items()},
            "messages_per_run": c1["42"]["messages"],
            "board": "100x100 torus (GameOfLifeLogic.fs:5), dotnet-mod2 seeds 0/1/42, 100 generations",
        },
        "fair_cpu": {
            "value": fair["cell_updates_per_s"] / 1e9,
            "unit": "GCUPS",
            "cores": threads,
            "kind": "port",
            "sample": f"bit-sliced carry-save stepper (oracle/gol_fast.c, AVX-512 build), {fair['width']}x"
            f"{fair['height']} torus splitmix 0x5EED, {fair['generations']} generations in {fair['seconds']:.1f} s",
        },
        "fair_cpu_all_cpus": None if fair_all is None else {
            "value": fair_all["cell_updates_per_s"] / 1e9,
            "unit": "GCUPS",
            "cores": avail,
            "sample": f"the same stepper on all {avail} available CPUs, {fair_all['generations']} generations in "
            f"{fair_all['seconds']:.1f} s",
        },
        "host": host,
    }


def _handle_run(args, W, H, boundary, devices, transport):
    """One handle-leg board: warmup passes, args.steps timed passes of its depth (host wall time around gol_step +
    gol_synchronize, and the library's own HIP events: gol_step_timed), then untimed to args.verify_gen and hashed."""
    from gameoflifewithactors_amd import Board

    parts = len(devices)
    with Board(W, H, boundary, devices=devices if parts > 1 else None) as b:
        if transport == "rccl":
            b.set_option("transport", 2)  # raises when RCCL cannot serve this placement
        k = b.parts()[0]["ghost"] if parts > 1 else b.info()["tblock_k"]
        b.seed_splitmix(args.seed)
        # warm up to the main leg's first timed generation: the same window of the same board (the launch time drifts
        # with the board's activity and the clock)
        b.step(max(args.warmup * k, args.handle_first_gen))
        b.synchronize()
        first = b.generation
        t0 = time.perf_counter()
        dev_us = b.step_timed(args.steps * k)
        dt = time.perf_counter() - t0
        timing = b.pass_timing() if parts > 1 else None
        out = {
            "value": round(W * H * args.steps * k / dt / 1e9, 3),
            "value_device_events": round(W * H * args.steps * k / (dev_us * 1e-6) / 1e9, 3),
            "unit": "GCUPS",
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "avg_pass_us_device_events": round(dev_us / args.steps, 2),
            "generations_per_step": k,
            "first_generation_timed": first,
            "transport": b.transport(),
        }
        if parts == 1:
            # the drop-in's own figure: the same algorithmic bytes per pass as the main
            # leg's roofline, over the library's HIP events around the C-ABI board's passes on /opt/rocm's runtime
            alg = 2 * W * H / 8
            pass_s = dev_us * 1e-6 / args.steps
            out["roofline"] = {"bound": "hbm", "achieved": round(alg / pass_s / 1e9, 2), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(alg / pass_s / 1e9 / HBM_PEAK_GBS, 4),
                               "alg_bytes_per_launch": alg, "avg_launch_us": round(pass_s * 1e6, 2),
                               "timing": "gol_step_timed: the library's HIP events on the board's stream"}
            slots = valu_slots_per_word_gen(b.info()["ilv"] or 1)
            vt = slots * (W * H / 32) * k / pass_s / 1e12
            out["roofline_valu"] = {"bound": "valu", "achieved": round(vt, 3), "peak": round(VALU_PEAK_TSLOTS, 2),
                                    "frac": round(vt / VALU_PEAK_TSLOTS, 4)}
        if timing is not None:
            out["pass_timing_us"] = timing
            out["edge_wait_us_max"] = max(t["edge_wait_us"] for t in timing)
        if args.verify_gen >= b.generation:
            b.step(args.verify_gen - b.generation)
            out["verify_generation"] = b.generation
            out["hash"] = b.hash()
            out["population"] = b.population()
    return out


def handle_leg(args, W, H, boundary, parts, ndev):
    """The one-process C-ABI board (what the F# drop-in calls: gol_create / gol_create_multi, csrc/gol_multi.cpp) on
    the bench board, in this child process WITHOUT torch, so the library runs on the HIP runtime it links
    (/opt/rocm), as the F# host does.  parts = 1: the single board; parts > 1: row strips on devices 0..parts-1
    (round-robin over the visible devices: a one-GPU box rehearses it with every strip on device 0), once with the
    default peer-copy transport and, when every strip has its own GPU, once more over RCCL.  Each run reports its
    rate and the board's hash at args.verify_gen (bench.py compares them with the main leg's)."""
    from gameoflifewithactors_amd import _lib

    devices = [i % ndev for i in range(parts)]
    out = {"strips": parts, "devices": devices, "hip_runtime": None,
           "rccl_possible": parts > 1 and len(set(devices)) == parts}
    # one transport per child process (run_handle_leg): an RCCL run that fails or hangs costs only itself
    runs = {"rccl": None} if args.handle_transport == "rccl" else {"single" if parts == 1 else "peer": None}
    for name in runs:
        try:
            runs[name] = _handle_run(args, W, H, boundary, devices, name)
        except Exception as e:  # noqa: BLE001 -- reported in the line, the main leg stands
            runs[name] = {"error": f"{type(e).__name__}: {e}"}
    out["hip_runtime"] = _lib.hip_runtimes()
    first = next(iter(runs))
    out.update({k: v for k, v in runs[first].items()})  # the default transport's figures at the top level
    out["runs"] = runs
    return out


def _handle_child(args, W, H, parts, verify_gen, first_gen, transport, timeout):
    cmd = [sys.executable, os.path.abspath(__file__), "--handle-leg-child", "--width", str(W), "--height", str(H),
           "--boundary", args.boundary, "--handle-parts", str(parts), "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--seed", str(args.seed), "--verify-gen", str(verify_gen),
           "--handle-first-gen", str(first_gen), "--handle-transport", transport]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
    env["WORLD_SIZE"] = "1"
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"handle leg ({transport}) exceeded {timeout:.0f} s (killed)"}
    if r.returncode != 0:
        return {"error": f"handle leg ({transport}) exited {r.returncode}: {r.stderr.strip()[-600:]}"}
    return json.loads(r.stdout.strip().splitlines()[-1])


def run_handle_leg(args, W, H, boundary, parts, verify_gen, first_gen=0):
    """The handle leg in child processes of rank 0, each under a time limit and never importing torch (bench.py
    main): the default transport first, then -- when every strip has its own GPU -- RCCL in a second child, since
    it creates a communicator over all GPUs inside one process and a failure or hang there must cost neither the
    main line nor the peer-copy figures."""
    del boundary
    out = _handle_child(args, W, H, parts, verify_gen, first_gen, "default", args.handle_timeout)
    if "error" in out or not out.get("rccl_possible"):
        return out
    rccl = _handle_child(args, W, H, parts, verify_gen, first_gen, "rccl", min(args.handle_timeout, 180.0))
    out.setdefault("runs", {})["rccl"] = rccl.get("runs", {}).get("rccl", rccl) if "error" not in rccl else rccl
    return out


def traffic_key(W, rows, boundary, k, ilv):
    return f"{W}x{rows}_{boundary}_k{k}_m{ilv}"


def load_traffic(path, key, fingerprint):
    """The PMC measurement for this configuration, only if it was taken on this build's device code."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    e = d.get(key)
    if not e or not fingerprint or e.get("device_code") != fingerprint:
        return None
    return e


def board_leg(args) -> dict:
    """BASELINE configs 1, 2 and 5 on the C-ABI board (what the F# drop-in calls): the board the reference seeds
    (--init), one gol_step call of --gens-per-step generations per step, so the engine picks the pass it picks for
    the size (single-wave, cooperative, LDS-resident or streaming).  Host wall time around the timed calls, and the
    device time of each call from the library's own HIP events (gol_step_timed).  N = 1 only.  This leg never imports
    torch: the library runs on the HIP runtime it links (/opt/rocm), as under the F# host, and no torch object
    outlives the board's stream (round 3's exit-time SIGSEGV: a torch ExternalStream around the board's stream,
    destroyed by gol_destroy while torch still held it).  The final board is checked against the
    golden_long.json checkpoint at its generation when one exists (configs 2 and 5)."""
    from gameoflifewithactors_amd import BOUNDED, INIT_DOTNET_MOD2, INIT_DOTNET_NEXT2, TORUS, Board, checkpoints, patterns

    W, H = args.width, args.height
    boundary = TORUS if args.boundary == "torus" else BOUNDED
    gps = args.gens_per_step or args.generations
    steps = args.steps if args.steps > 0 else 1
    with Board(W, H, boundary) as b:
        if args.init == "dotnet-mod2":
            b.seed_dotnet(args.seed, INIT_DOTNET_MOD2)
        elif args.init == "dotnet-next2":
            b.seed_dotnet(args.seed, INIT_DOTNET_NEXT2)
        elif args.init.startswith("rle:"):
            for text, x, y in patterns.parse_placements(args.init[4:]):
                b.place_rle(text, x, y)
        else:
            raise SystemExit(f"unknown --init {args.init}")
        h0, p0 = b.hash(), b.population()
        for _ in range(args.warmup):
            b.step(gps)
        b.synchronize()
        first = b.generation
        dev_us = 0.0
        t0 = time.perf_counter()
        for _ in range(steps):
            dev_us += b.step_timed(gps)
        dt = time.perf_counter() - t0
        kernel_s = dev_us * 1e-6
        info = b.info()
        end_hash, pop = b.hash(), b.population()
        gens = steps * gps
        end_gen = b.generation
    name, case = checkpoints.board_case(W, H, boundary, args.init, args.seed)
    init_mark = checkpoints.initial_mark(case)
    verify = checkpoints.verdict(end_gen, end_hash, pop, checkpoints.at_generation(case, end_gen),
                                 f"tests/golden/golden_long.json[{name}]" if name else None)
    if init_mark is not None:
        verify["initial_ok"] = (h0, p0) == tuple(init_mark)
        # ok is True only when an end-state comparison passed: with no checkpoint at the end
        # generation the final board was not compared, so a matching initial board leaves it None
        if not verify["initial_ok"]:
            verify["ok"] = False
    return {
        "metric": "cell updates/sec (GCUPS) of gol_step on the C-ABI board",
        "value": round(W * H * gens / dt / 1e9, 3),
        "unit": "GCUPS",
        "n_gpus": 1,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / steps * 1e3, 4),
        "us_per_generation": round(dt / gens * 1e6, 4),
        "us_per_generation_kernel": round(kernel_s / gens * 1e6, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (bit-packed cells)" if info["packed"] else "u8 (byte cells)",
        "data": f"synthetic ({args.init}, seed {args.seed})",
        "config": {"workload": f"{W}x{H} {args.boundary} board, {args.init} seed {args.seed}, {gens} generations "
                               f"timed in {steps} gol_step call(s)",
                   "width": W, "height": H, "boundary": args.boundary, "init": args.init, "seed": args.seed,
                   "generations_per_step": gps, "first_generation_timed": first, "generations_timed": gens,
                   "tblock_k": info["tblock_k"], "interleave": info["ilv"], "parallelism": "single board",
                   "initial_hash": f"{h0:016x}", "final_hash": f"{end_hash:016x}", "final_population": pop},
        "verify": verify,
        "hip_runtime": _lib_runtimes(),
    }


def _lib_runtimes():
    from gameoflifewithactors_amd import _lib

    return _lib.hip_runtimes()


def main():
    args = parse()
    if args.handle_leg_child:  # rank 0's child process (run_handle_leg): no torch, the library's own runtime
        from gameoflifewithactors_amd import TORUS, BOUNDED, _lib

        boundary = TORUS if args.boundary == "torus" else BOUNDED
        print(json.dumps(handle_leg(args, args.width, args.height, boundary, args.handle_parts,
                                    _lib.device_count())), flush=True)
        return
    if args.init != "splitmix":
        if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
            raise SystemExit("--init other than splitmix times the single C-ABI board (N = 1)")
        line = board_leg(args)
        print(json.dumps(line), flush=True)
        if line["verify"]["ok"] is False:
            raise SystemExit("board differs from the golden checkpoint (verify.ok false)")
        return
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
    host_group = None
    if world > 1:
        # a mis-paired exchange or a dead peer ends the run with an error after this long instead of hanging
        timeout = datetime.timedelta(seconds=120)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev), timeout=timeout)
            # host-side barrier for the handle leg: the waiting ranks must not keep an RCCL kernel spinning
            # on the devices rank 0's one-process board is running on
            host_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=max(
                120, args.handle_timeout + min(args.handle_timeout, 180.0) + 60)))
        else:
            dist.init_process_group("gloo", timeout=timeout)
            host_group = dist.group.WORLD

    from gameoflifewithactors_amd import TORUS, BOUNDED, checkpoints
    from gameoflifewithactors_amd.strips import StripRunner

    from gameoflifewithactors_amd import _lib

    boundary = TORUS if args.boundary == "torus" else BOUNDED
    if args.board:
        args.width, args.height = args.board, args.board // world  # rows per GPU (last rank may own more)
        W, H = args.board, args.board
    else:
        W, H = args.width, args.height * world
    lib = _lib.load()
    ilv, kdef = default_layout(lib, W, args.height, boundary)  # rows per rank
    if args.ilv:
        ilv, kdef = args.ilv, int(lib.gol_default_tblock(args.ilv))  # (--tblock still sets the depth)
    # Temporal depth: --tblock, the engine default (--no-autotune), or by default a short on-box race between the depths
    # that are within a few percent of each other across MI355X boxes.
    if args.tblock:
        cands = [args.tblock]
    elif not args.no_autotune:
        cands = AUTOTUNE.get(ilv, [kdef])
    else:
        cands = [kdef]
    runner = StripRunner(W, H, boundary, max(cands), rank=rank, world=world, device=torch.device("cuda", dev), ilv=ilv)
    runner.seed_splitmix(args.seed)
    k, tune = cands[0], None
    if len(cands) > 1:
        # interleaved rounds (the board and the clock drift during the race), best round per depth
        per_gen = [float("inf")] * len(cands)
        for _ in range(3):
            for i, kk in enumerate(cands):
                runner.step_pass(kk)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(runner.compute_stream)
                for _ in range(2):
                    runner.step_pass(kk)
                e1.record(runner.compute_stream)
                torch.cuda.synchronize()
                per_gen[i] = min(per_gen[i], e0.elapsed_time(e1) / (2 * kk))
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
    first_gen = runner.generation  # generations the board has advanced before the timed window (race + warmup)
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

    # N > 1: the ranks, their GPUs, RCCL's view of the group and the main leg's per-rank halo figures, after the
    # timed region (every rank takes part)
    multi = multi_gpu_report(runner, dev, args.dist_backend, host_group) if world > 1 else None

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
    fingerprint = _lib.device_code_fingerprint(kernel=hot_kernel_symbol(ilv, k))
    tkey = traffic_key(W, args.height, args.boundary, k, ilv)
    tr = (load_traffic(args.traffic_json, tkey, fingerprint) or {}) if world == 1 else {}
    traffic = tr.get("bytes_per_launch")  # measured HBM bytes per launch (rocprofv3 PMC, calibrated)

    # Self-check (untimed, after every timed and reference leg): step on to the first committed golden checkpoint
    # at or after the generation the board reached and compare the all-reduced canonical hash and population
    # (gameoflifewithactors_amd/checkpoints.py); every rank takes part in the reductions.
    verify = None
    verify_gen = -1
    expected, source = None, None
    got_hash = got_pop = None
    if not args.no_verify:
        cname, case = checkpoints.splitmix_case(W, H, boundary, args.seed)
        expected = checkpoints.next_checkpoint(case, runner.generation)
        source = f"tests/golden/golden_full.json[{cname}]" if expected else None
        verify_gen = expected[0] if expected else runner.generation
        runner.step(verify_gen - runner.generation)
        torch.cuda.synchronize()
        got_hash, got_pop = runner.hash(), runner.population()
    runner.close()  # the main leg is done: its buffers go and its engine releases the library (_lib.unload-able)

    # One-process C-ABI leg (rank 0), after the main leg; the other ranks wait on a host barrier.
    parts = args.handle_parts if args.handle_parts >= 0 else world
    handle = None
    if parts >= 1:
        if world > 1:
            torch.cuda.synchronize()
            dist.barrier(group=host_group)
        if rank == 0:
            handle = run_handle_leg(args, W, H, boundary, parts, verify_gen, first_gen)
        if world > 1:
            dist.barrier(group=host_group)
    if rank == 0 and got_hash is not None:
        others = {}
        for name, run in ((handle or {}).get("runs") or {}).items():
            if isinstance(run, dict) and run.get("verify_generation") == verify_gen:
                others[f"handle_leg.{name}"] = run.get("hash")
        verify = checkpoints.verdict(verify_gen, got_hash, got_pop, expected, source, others)

    result = None
    if rank == 0:
        result = {
            "metric": "cell updates/sec (GCUPS), whole job over all GPUs, 65536^2 cells per GPU; % of HBM peak BW",
            "value": round(gcups, 3),
            "value_per_gpu": round(gcups / world, 3),
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
                "first_generation_timed": first_gen,
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
                "traffic_source": (f"profiles/pmc_traffic.json[{tkey}] (tools/pmc_traffic.sh), measured on this "
                                   f"build's device code {fingerprint}") if traffic else
                (f"no PMC measurement of {tkey} on this build's device code ({fingerprint})" if world == 1 else
                 "PMC traffic is measured at N = 1 only"),
                "kernel": kernel_name(ilv, k),
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
            "hip_runtime": _lib.hip_runtimes(),
            "device_code": fingerprint,
        }
        if multi is not None:
            result["multi_gpu"] = multi
        if verify is not None:
            result["verify"] = verify
        if handle is not None:
            result["handle_leg"] = handle
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N = 1 figure (rank 0 only)
            result["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if verify is not None and verify["ok"] is False:
        raise SystemExit("the timed board differs from its reference (verify.ok false)")


if __name__ == "__main__":
    main()
