"""Where the time of one reference-size gol_step call goes (BASELINE config 1: 100^2 torus, 100 generations):
host wall time of step + synchronize, the kernel alone (HIP events on the board's stream), and the wall time
of step + synchronize with the synchronize done by polling hipStreamQuery.  Prints one JSON line per variant."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gameoflifewithactors_amd import Board  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
gens = 100
with Board(100, 100, 0) as b:
    b.seed_dotnet(42)
    b.step(gens)
    b.synchronize()
    s = torch.cuda.ExternalStream(b.stream)
    for rep in range(3):
        wall, kern, spin = [], [], []
        for _ in range(50):
            t0 = time.perf_counter()
            b.step(gens)
            b.synchronize()
            wall.append(time.perf_counter() - t0)
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            b.step(gens)
            e1.record(s)
            e1.synchronize()
            kern.append(e0.elapsed_time(e1) / 1e3)
        for _ in range(50):
            t0 = time.perf_counter()
            b.step(gens)
            while hip.hipStreamQuery(ctypes.c_void_p(b.stream)) != 0:
                pass
            spin.append(time.perf_counter() - t0)
        med = lambda v: sorted(v)[len(v) // 2] * 1e6 / gens  # noqa: E731
        print(json.dumps({"rep": rep, "us_per_gen_wall": round(med(wall), 3), "us_per_gen_kernel": round(med(kern), 3),
                          "us_per_gen_wall_spin": round(med(spin), 3)}), flush=True)
