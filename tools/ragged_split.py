"""Pair-split sweep for a ragged board on the streaming pass (block rows), interleaved rounds.  Timing: gol_step_timed
after 40 warm-up generations, as tools/ragged_stream_ab.py.

    python tools/ragged_split.py [--board WxHxB] [--gens G] [--splits 0.56,0.60,...] [--rounds N]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--board", default="65535x65535x1")
    p.add_argument("--gens", type=int, default=48)
    p.add_argument("--splits", default="0.56,0.60,0.64,0.68,0.72")
    p.add_argument("--rounds", type=int, default=2)
    a = p.parse_args()
    from gameoflifewithactors_amd import Board

    w, h, boundary = (int(x) for x in a.board.split("x"))
    for rep in range(a.rounds):
        for sp in (float(x) for x in a.splits.split(",")):
            with Board(w, h, boundary, options={"split": int(sp * 65536)}) as b:
                b.seed_splitmix(0x5EED)
                b.step(40)
                b.synchronize()
                us = b.step_timed(a.gens) / a.gens
                hsh = b.hash()
            print(json.dumps({"rep": rep, "board": a.board, "split": sp, "us_per_gen": round(us, 3),
                              "hash": f"{hsh:016x}"}), flush=True)


if __name__ == "__main__":
    main()
