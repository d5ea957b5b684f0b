"""One rank's pass of the N > 1 path, alone on one GPU: rank 0 of a LocalBoard of `--strips` ghost-row strips
(65536 x 65536 per strip by default), its halo copied from the (idle) neighbour strips, timed phase by phase
(StripRunner.timed_pass: interior launch end, edge-band release, edge bands' end) for several caps on the waves held
back from the interior launch for the edge bands (StripRunner.spare_cap; "none" = the runner's own plan), interleaved.
Against the single board's pass on the same box (world 1).  Timing only: the neighbours do not step.

    python tools/strip_pass_probe.py [--strips 2] [--passes 6] [--caps none,0,32,64,128]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=65536)
    p.add_argument("--rows", type=int, default=65536)
    p.add_argument("--strips", type=int, default=2)
    p.add_argument("--passes", type=int, default=6)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--caps", default="none,0,16,32,64,128")
    a = p.parse_args()
    import torch

    from gameoflifewithactors_amd.strips import LocalBoard, StripRunner

    caps = [None if c == "none" else int(c) for c in a.caps.split(",")]
    single = StripRunner(a.width, a.rows, 0, 32, ilv=4)
    single.seed_splitmix(0x5EED)
    for _ in range(5):
        single.step_pass()
    with LocalBoard(a.width, a.rows * a.strips, 0, 32, a.strips, ilv=4) as lb:
        lb.seed_splitmix(0x5EED)
        lb.step(160)
        r = lb.runners[0]
        torch.cuda.synchronize()
        for rnd in range(a.rounds):
            ts = []
            for _ in range(a.passes):
                ts.append(single.timed_pass()["interior_us"])
            print(json.dumps({"round": rnd, "what": "single board", "pass_us": round(statistics.median(ts), 1)}),
                  flush=True)
            for cap in caps:
                r.spare_cap = cap
                rows = [r.timed_pass() for _ in range(a.passes)]
                med = {k: round(statistics.median(x[k] for x in rows), 1) for k in rows[0]}
                med["pass_us"] = max(med["interior_us"], med.get("edge_done_us", 0))
                print(json.dumps({"round": rnd, "what": f"rank 0 of {a.strips}", "spare_cap": cap, **med}), flush=True)
    single.close()


if __name__ == "__main__":
    main()
