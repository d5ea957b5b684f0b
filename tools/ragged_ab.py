"""Ragged byte boards (width not a multiple of 32, beyond the single-wave pass): the cooperative pass through
whole-word scratch rows (option coop=1) against the per-generation byte step (coop=0), interleaved, host wall
time around one gol_step call + gol_synchronize.  One JSON line per (board, pass, round)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gameoflifewithactors_amd import Board  # noqa: E402

BOARDS = [(255, 257, 2000), (1001, 1001, 1000), (2049, 2049, 1000), (4095, 4095, 500), (8191, 4000, 300)]
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for (w, h, gens) in BOARDS:
        for mode in ("1", "0"):
            with Board(w, h, 0, options={"coop": int(mode)}) as b:
                b.seed_dotnet(42)
                b.step(20)
                b.synchronize()
                t0 = time.perf_counter()
                b.step(gens)
                b.synchronize()
                dt = time.perf_counter() - t0
            print(json.dumps({"rep": rep, "w": w, "h": h, "gens": gens, "pass": "coop" if mode == "1" else "bytestep",
                              "us_per_gen": round(dt / gens * 1e6, 3)}), flush=True)
