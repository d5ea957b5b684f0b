"""Sweep temporal-block depth k (and optionally segment rows) on one GPU; prints one JSON line per config.

    python tools/sweep.py --size 65536 --ks 1,2,4,8,16,24,32 --passes 8
Timing: the library's own HIP events around `passes` launches (gol_step_timed, after 2 warm-up launches); no torch.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--height", type=int, default=0)
    p.add_argument("--ks", default="1,2,4,8,16,24,32")
    p.add_argument("--passes", type=int, default=8)
    p.add_argument("--boundary", type=int, default=0)
    p.add_argument("--ilv", type=int, default=0, help="packed layout (0 = the engine default for the width)")
    p.add_argument("--split", type=float, default=None, help="board option 'split' (fraction; negative = off)")
    p.add_argument("--split2", type=float, default=None, help="board option 'split2' (fraction, three-wave groups)")
    p.add_argument("--seam", type=int, default=0, help="board option 'seam' (0 = engine choice, -1 = halo-lane strips)")
    p.add_argument("--pre", type=int, default=0, help="generations stepped before the timed passes (bench.py's window "
                   "starts at generation 312)")
    a = p.parse_args()
    from gameoflifewithactors_amd import Board, _lib

    W = a.size
    H = a.height or a.size
    lib = _lib.load()
    ilv = a.ilv or lib.gol_default_ilv(W)
    opts = {"coop": 0, "seam": a.seam}
    if a.split is not None:
        opts["split"] = int(a.split * 65536) if a.split >= 0 else -1
    if a.split2 is not None:
        opts["split2"] = int(a.split2 * 65536)
    for k in [int(x) for x in a.ks.split(",")]:
        if not lib.gol_supported_k(k, ilv):
            continue
        with Board(W, H, a.boundary, tblock_k=k, ilv=ilv, options=opts) as b:
            b.seed_splitmix(0x5EED)
            b.step(2 * k + a.pre)
            b.synchronize()
            t = b.step_timed(a.passes * k) / 1e6 / a.passes
            h = b.hash()
            gcups = W * H * k / t / 1e9
            print(json.dumps({"W": W, "H": H, "ilv": ilv, "k": k, "seam": a.seam, "split": a.split, "split2": a.split2, "pre": a.pre, "us_per_pass": round(t * 1e6, 1), "gcups": round(gcups, 1),
                              "alg_GBps": round(W * H / 4 / t / 1e9, 1), "hash": f"{h:016x}",
                              }), flush=True)


if __name__ == "__main__":
    main()
