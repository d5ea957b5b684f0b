"""Interleaved A/B of the byte-board passes (ragged widths the single-wave pass does not take): LDS-resident
(GOL_RESIDENT_MAX_CELLS=65536) against the per-generation byte step (GOL_RESIDENT_MAX_CELLS=0), same process,
`reps` rounds.  Host wall time around gol_step + gol_synchronize; prints one JSON line per (board, pass, round)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gameoflifewithactors_amd import Board  # noqa: E402

BOARDS = [(129, 127), (181, 90), (255, 64), (300, 54), (200, 100), (181, 181), (255, 257)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
gens = 2000
os.environ["GOL_WAVE_RESIDENT"] = "0"
for rep in range(reps):
    for (w, h) in BOARDS:
        for mode, cells in (("resident", "65536"), ("bytestep", "0")):
            os.environ["GOL_RESIDENT_MAX_CELLS"] = cells
            with Board(w, h, 0) as b:
                b.seed_dotnet(42)
                b.step(2)
                b.synchronize()
                t0 = time.perf_counter()
                b.step(gens)
                b.synchronize()
                dt = time.perf_counter() - t0
            print(json.dumps({"rep": rep, "w": w, "h": h, "cells": w * h, "pass": mode,
                              "us_per_gen": round(dt / gens * 1e6, 3)}), flush=True)
