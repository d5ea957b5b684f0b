"""Cooperative pass (csrc/gol_coop.hip) option sweep on BASELINE config 2 (4096^2 torus, dotnet-mod2 seed 42,
1000 generations per gol_step call).  Timing: HIP events on the board's stream around one call, after one warm call.
One JSON line per (round, option set).

    python tools/coop_sweep.py [--rounds 2] [--size 4096] [--boundary 0] coop_k=6,8,10 coop_poll_delay=0,8,16
"""
import argparse
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--size", type=int, default=4096)
    p.add_argument("--boundary", type=int, default=0)
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("grid", nargs="*", help="option=v1,v2,... (board options, gol_set_option)")
    a = p.parse_args()
    import torch

    from gameoflifewithactors_amd import Board

    names = [g.split("=")[0] for g in a.grid]
    values = [[int(v) for v in g.split("=")[1].split(",")] for g in a.grid]
    for rep in range(a.rounds):
        for combo in itertools.product(*values) if values else [()]:
            opts = dict(zip(names, combo))
            with Board(a.size, a.size, a.boundary, options=opts) as b:
                b.seed_dotnet(42)
                s = torch.cuda.ExternalStream(b.stream)
                b.step(a.gens)
                b.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                b.step(a.gens)
                e1.record(s)
                b.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.gens
                h = b.hash()
            print(json.dumps({"rep": rep, "size": a.size, "boundary": a.boundary, "options": opts,
                              "us_per_gen": round(us, 4), "hash_after": h}), flush=True)


if __name__ == "__main__":
    main()
