"""A/B of the mid-size passes, interleaved on one box: the cooperative band pass (gol_coop.hip) against the
rows-on-lanes band pass (gol_lanes.hip) at several window widths and depths.  Timing: the library's own HIP events
around one gol_step call (gol_step_timed; no torch in the process) after a warm-up call.  One JSON line per (board,
variant, round), with the board's hash so the variants can be seen to agree.

    python tools/lanes_ab.py [--rounds N] [--boards WxHxB,...] [--gens G] [--variants coop,l9,l5,l17,l9k6,...]

A board WxHxB: B = 0 torus, 1 bounded.  Variant names: "coop" (k = default), "coopkN", "coopc" (launched by
hipLaunchCooperativeKernel: board option coop_launch 1), "coopdD" (poll delay D); "lM" (lanes, m = M) and "lMkN" (depth N), "lMdD" (poll
delay D).
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BOARDS = "4096x4096x0,4096x4096x1,2048x2048x0,8192x4096x0,1024x1024x0"
VARIANTS = "coop,l9,l5,l17,l9k6,l9k10,l5k10"


def options(name):
    m = re.fullmatch(r"coop(c?)(?:k(\d+))?(?:d(\d+))?", name)
    if m:
        o = {"lanes": 0, "coop_launch": 1 if m.group(1) else 0}
        if m.group(2):
            o["coop_k"] = int(m.group(2))
        if m.group(3):
            o["coop_poll_delay"] = int(m.group(3))
        return o
    m = re.fullmatch(r"l(\d+)(?:k(\d+))?(?:d(\d+))?", name)
    if not m:
        raise SystemExit(f"unknown variant {name}")
    o = {"lanes": 1, "lanes_m": int(m.group(1))}
    if m.group(2):
        o["coop_k"] = int(m.group(2))
    if m.group(3):
        o["coop_poll_delay"] = int(m.group(3))
    return o


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--boards", default=BOARDS)
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--variants", default=VARIANTS)
    a = p.parse_args()
    from gameoflifewithactors_amd import INIT_DOTNET_MOD2, Board

    boards = [tuple(int(x) for x in s.split("x")) for s in a.boards.split(",")]
    for rep in range(a.rounds):
        for (w, h, boundary) in boards:
            for name in a.variants.split(","):
                try:
                    with Board(w, h, boundary, options=options(name)) as b:
                        b.seed_dotnet(42, INIT_DOTNET_MOD2)
                        b.step(a.gens)
                        b.synchronize()
                        us = b.step_timed(a.gens) / a.gens
                        lanes = b.get_option("lanes_launches")
                        hsh = b.hash()
                except Exception as e:  # noqa: BLE001 -- a variant that does not apply to the board
                    print(json.dumps({"rep": rep, "w": w, "h": h, "boundary": boundary, "variant": name,
                                      "error": str(e)[:160]}), flush=True)
                    continue
                print(json.dumps({"rep": rep, "w": w, "h": h, "boundary": boundary, "variant": name,
                                  "us_per_gen": round(us, 4), "lanes_launches": lanes, "hash": f"{hsh:016x}"}),
                      flush=True)


if __name__ == "__main__":
    main()
