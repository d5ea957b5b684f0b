"""Does the step kernel's speed depend on the board's contents?  The instruction stream is data-independent,
so a difference means the clock moves with switching activity (power limit).  65536^2, default depth:
an all-dead board, a fresh 50 % random board, and the same random board after 2000 generations."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from gameoflifewithactors_amd import Board

    n = 65536
    with Board(n, n) as b:
        k = b.info()["tblock_k"]
        s = torch.cuda.ExternalStream(b.stream)

        def timed(label, passes=8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            b.step(passes * k)
            e1.record(s)
            b.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / passes
            print(json.dumps({"board": label, "k": k, "us_per_pass": round(us, 1),
                              "gcups": round(n * n * k / us / 1e3, 1), "population": b.population()}), flush=True)

        for rep in range(2):
            b.clear()
            timed(f"dead#{rep}")
            b.seed_splitmix(0x5EED + rep)
            timed(f"random50#{rep}", passes=2)
            b.step(2000 - 2 * k)
            timed(f"random50+2000gen#{rep}")


if __name__ == "__main__":
    main()
