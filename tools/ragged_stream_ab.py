"""Ragged boards past the cooperative pass (width not a multiple of 32, wider than 8192 or above 2^26 cells), passes
interleaved on one box: block rows in the aligned layouts (board option ragged_ring=2: ring rows on a torus,
column-masked rows when bounded), the ilv-1 rows (ragged_ring=0), the default choice by size (auto, ragged_ring=1),
and optionally the per-generation byte step
(ragged_stream=0).  Timing: the
library's own HIP events around one gol_step call (gol_step_timed; no torch in the process), after 40 warm-up
generations; the state stays in the scratch rows between the calls (DESIGN.md 4.1 "Ragged rows").  One JSON line per
(board, boundary, pass, depth, round).

    python tools/ragged_stream_ab.py [--rounds N] [--boards WxHxG,...] [--ks 0,8,16] [--passes ring,m1,bytestep]

--ks: the boards' tblock_k (0 = the engine default).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BOARDS = "10001x10001x192,16383x16383x96,8193x20000x192,65535x65535x48"
OPTS = {"ring": {"ragged_stream": 1, "ragged_ring": 2}, "m1": {"ragged_stream": 1, "ragged_ring": 0},
        "auto": {"ragged_stream": 1, "ragged_ring": 1},
        "bytestep": {"ragged_stream": 0}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--boards", default=BOARDS)
    p.add_argument("--ks", default="0")
    p.add_argument("--boundaries", default="0,1")
    p.add_argument("--passes", default="ring,m1")
    a = p.parse_args()
    from gameoflifewithactors_amd import Board

    boards = [tuple(int(x) for x in s.split("x")) for s in a.boards.split(",")]
    for rep in range(a.rounds):
        for (w, h, gens) in boards:
            for boundary in (int(x) for x in a.boundaries.split(",")):
                for k in (int(x) for x in a.ks.split(",")):
                    for name in a.passes.split(","):
                        g = gens if name != "bytestep" else max(4, gens // 10)
                        with Board(w, h, boundary, tblock_k=k, options=OPTS[name]) as b:
                            b.seed_splitmix(0x5EED)
                            b.step(40)
                            b.synchronize()
                            us = b.step_timed(g) / g
                            info = b.info()
                            h_ = b.hash()
                        print(json.dumps({"rep": rep, "w": w, "h": h, "boundary": boundary, "gens": g, "pass": name,
                                          "tblock_k": info["tblock_k"], "us_per_gen": round(us, 3),
                                          "gcups": round(w * h / us / 1e3, 1), "hash": f"{h_:016x}"}), flush=True)


if __name__ == "__main__":
    main()
