"""Throughput of the one-process multi-GPU board (gol_create_multi) against the single board, on one GPU.

All strips share device 0 here, so the total rate should match the single board's: the difference is the
cost of the strip protocol (ghost-row kernel variant, two edge-band launches and two peer copies per strip
per pass).  On a node, devices=range(n) puts one strip per GPU.

    python tools/multi_bench.py --size 65536 --parts 1,2,4,8 --passes 16 [--weak]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--parts", default="1,2,4,8")
    p.add_argument("--passes", type=int, default=16)
    p.add_argument("--generations", type=int, default=0, help="time this many generations instead of --passes")
    p.add_argument("--tblock", type=int, default=0)
    p.add_argument("--weak", action="store_true", help="board height = size * parts (each strip size x size)")
    p.add_argument("--devices", default="", help="comma list of devices per part (default: all on device 0)")
    a = p.parse_args()
    from gameoflifewithactors_amd import Board

    n_side = a.size
    for n in [int(x) for x in a.parts.split(",")]:
        devs = [int(x) for x in a.devices.split(",")][:n] if a.devices else [0] * n
        kw = {"devices": devs} if n > 1 else {}
        height = n_side * n if a.weak else n_side
        with Board(n_side, height, 0, tblock_k=a.tblock, **kw) as b:
            k = b.info()["tblock_k"]
            k = min(k, min(pt["ghost"] for pt in b.parts())) if n > 1 else k
            b.seed_splitmix(0x5EED)
            b.step(2 * k)
            b.synchronize()
            if a.generations:
                a.passes = -(-a.generations // k)
            t0 = time.perf_counter()
            b.step(a.passes * k)
            b.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"parts": n, "devices": devs if n > 1 else [b.parts()[0]["device"]], "k": k,
                              "size": [n_side, height], "ms_per_pass": round(dt / a.passes * 1e3, 4),
                              "gcups": round(n_side * height * a.passes * k / dt / 1e9, 1),
                              "hash": b.hash()}), flush=True)


if __name__ == "__main__":
    main()
