"""Generate the golden fixtures in tests/golden/ from the CPU oracle (oracle/gol_oracle.{c,py}).

The reference ships no fixtures and cannot run here (see DESIGN.md "Parity"), so every vector below is
produced by the oracle restatement, whose own pins (published .NET Random values, Life known answers,
the actor-protocol restatement) are checked in tests/test_oracle.py.

    python tests/golden/make_golden.py            # small fixtures (seconds)

Outputs:
    golden_small.json   hashes / populations at checkpoints for each case
    golden_boards.npz   bit-packed boards (np.packbits, little bit order, row-major [y, x])
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gol_oracle as o  # noqa: E402


def pack(b: np.ndarray) -> np.ndarray:
    return np.packbits(b, axis=None, bitorder="little")


def checkpoints(board, gens, boundary, cps):
    out = {}
    cur = board
    done = 0
    for cp in sorted(cps):
        cur = o.c_run(cur, cp - done, boundary)
        done = cp
        out[str(cp)] = {"hash": str(o.c_hash(cur)), "population": o.population(cur)}
    return out, cur


def main():
    cases = {}
    boards = {}

    # C1: the reference's default board (GameOfLifeLogic.fs:5), torus, dotnet-mod2 init, 100 generations
    for seed in (0, 1, 42):
        b0 = o.seed_dotnet(100, 100, seed, 0)
        cps, b100 = checkpoints(b0, 100, o.TORUS, [0, 1, 2, 10, 100])
        name = f"c1_torus100_dotnetmod2_seed{seed}"
        cases[name] = {"width": 100, "height": 100, "boundary": "torus", "init": "dotnet-mod2", "seed": seed,
                       "checkpoints": cps}
        boards[name + "_g0"] = pack(b0)
        boards[name + "_g100"] = pack(b100)

    # Script.fsx: bounded 256x256, Next 2 = 0 init
    b0 = o.seed_dotnet(256, 256, 7, 1)
    cps, bend = checkpoints(b0, 500, o.BOUNDED, [0, 1, 10, 100, 500])
    cases["script_bounded256_dotnetnext2_seed7"] = {"width": 256, "height": 256, "boundary": "bounded",
                                                    "init": "dotnet-next2", "seed": 7, "checkpoints": cps}
    boards["script_bounded256_dotnetnext2_seed7_g500"] = pack(bend)

    # splitmix init on a ragged packed size, both boundaries
    for bname, bd in (("torus", o.TORUS), ("bounded", o.BOUNDED)):
        b0 = o.seed_splitmix(320, 77, 0x5EED)
        cps, bend = checkpoints(b0, 200, bd, [0, 1, 33, 200])
        name = f"splitmix_{bname}_320x77"
        cases[name] = {"width": 320, "height": 77, "boundary": bname, "init": "splitmix", "seed": 0x5EED,
                       "checkpoints": cps}
        boards[name + "_g200"] = pack(bend)

    # patterns (C5 shapes at fixture-friendly sizes)
    for bname, bd, n in (("bounded", o.BOUNDED, 256), ("torus", o.TORUS, 256)):
        b0 = np.zeros((n, n), np.uint8)
        o.place_rle(b0, o.GOSPER_GUN, 10, 10)
        o.place_rle(b0, o.R_PENTOMINO, 180, 150)
        cps, bend = checkpoints(b0, 2000, bd, [0, 30, 100, 1000, 2000])
        name = f"gun_rpent_{bname}{n}"
        cases[name] = {"width": n, "height": n, "boundary": bname, "init": "rle",
                       "rle": [["gosper_gun", 10, 10], ["r_pentomino", 180, 150]], "checkpoints": cps}
        boards[name + "_g2000"] = pack(bend)

    with open(os.path.join(HERE, "golden_small.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (CPU oracle)", "cases": cases}, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "golden_boards.npz"), **boards)
    print(f"wrote {len(cases)} cases, {len(boards)} boards")


if __name__ == "__main__":
    main()
