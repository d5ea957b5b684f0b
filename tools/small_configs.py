"""Wall time of gol_step on the reference-size boards (BASELINE configs 1, 2, 5 and small-board sweep).
Arguments: board options name=value (gol_set_option, e.g. resident_max_cells=0 wave_resident=0 coop=0; none: the
default cut-overs); every line records them."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gameoflifewithactors_amd import Board

CASES = [(100, 100, 0, 100, 'dotnet'), (100, 100, 0, 10000, 'dotnet'), (100, 100, 1, 10000, 'dotnet'),
         (64, 64, 0, 20000, 'dotnet'), (128, 128, 1, 20000, 'dotnet'), (96, 192, 0, 20000, 'dotnet'), (4096, 4096, 0, 1000, 'dotnet'),
         (256, 256, 1, 100000, 'rle'), (128, 128, 0, 20000, 'dotnet'), (256, 256, 0, 20000, 'dotnet'),
         (512, 256, 0, 10000, 'dotnet'), (512, 512, 0, 10000, 'dotnet'), (1024, 512, 0, 10000, 'dotnet'), (1024, 1024, 0, 10000, 'dotnet'),
         (2048, 2048, 0, 4000, 'dotnet'), (4096, 4096, 1, 1000, 'dotnet'), (8192, 4096, 0, 1000, 'dotnet'),
         (255, 257, 0, 10000, 'dotnet')]
opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[1:]}
for (w, h, bnd, gens, seed) in CASES:
    with Board(w, h, bnd, options=opts) as b:
        if seed == 'dotnet':
            b.seed_dotnet(42)
        else:
            b.place_rle("b2o$2o$bo!", w // 2, h // 2)
        b.step(2); b.synchronize()
        t0 = time.perf_counter(); b.step(gens); b.synchronize(); dt = time.perf_counter() - t0
        print(json.dumps({"options": opts, "w": w, "h": h, "boundary": bnd, "gens": gens,
                          "ms": round(dt * 1e3, 3), "us_per_gen": round(dt / gens * 1e6, 3),
                          "gcups": round(w * h * gens / dt / 1e9, 2), "k": b.info()["tblock_k"]}), flush=True)
