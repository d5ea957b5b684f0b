"""Ragged boards past the cooperative pass (width not a multiple of 32, wider than 8192 or above 2^26 cells): the
streaming pass on whole-word scratch rows (board option ragged_stream=1, the default) against the per-generation
byte step (ragged_stream=0), interleaved, on both boundaries.  Timing: HIP events on the board's stream around one
gol_step call (the board is warmed by 40 generations first).  One JSON line per (board, boundary, pass, depth, round).

    python tools/ragged_stream_ab.py [--rounds N] [--boards WxHxG,...] [--ks 0,8,16] [--no-bytestep]

--ks: the boards' tblock_k (0 = the engine default).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BOARDS = "10001x10001x200,16383x16383x100,8193x20000x200,65535x65535x48"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--boards", default=BOARDS)
    p.add_argument("--ks", default="0")
    p.add_argument("--boundaries", default="0,1")
    p.add_argument("--no-bytestep", action="store_true")
    a = p.parse_args()
    import torch

    from gameoflifewithactors_amd import Board

    boards = [tuple(int(x) for x in s.split("x")) for s in a.boards.split(",")]
    for rep in range(a.rounds):
        for (w, h, gens) in boards:
            for boundary in (int(x) for x in a.boundaries.split(",")):
                for k in (int(x) for x in a.ks.split(",")):
                    for stream in ((1,) if a.no_bytestep else (1, 0)):
                        g = gens if stream else max(4, gens // 10)
                        with Board(w, h, boundary, tblock_k=k, options={"ragged_stream": stream}) as b:
                            b.seed_splitmix(0x5EED)
                            s = torch.cuda.ExternalStream(b.stream)
                            b.step(40)
                            b.synchronize()
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record(s)
                            b.step(g)
                            e1.record(s)
                            b.synchronize()
                            us = e0.elapsed_time(e1) * 1e3 / g
                            info = b.info()
                        print(json.dumps({"rep": rep, "w": w, "h": h, "boundary": boundary, "gens": g,
                                          "pass": "stream" if stream else "bytestep", "tblock_k": info["tblock_k"],
                                          "us_per_gen": round(us, 3), "gcups": round(w * h / us / 1e3, 1)}),
                              flush=True)


if __name__ == "__main__":
    main()
