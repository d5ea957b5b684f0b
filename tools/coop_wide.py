"""Cooperative pass vs streaming on 8192-wide boards around the 2^25-cell cut-over (A/B timing).
python tools/coop_wide.py  -- run under GOL_ILV / GOL_COOP / GOL_COOP_MAX_CELLS settings; prints JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gameoflifewithactors_amd import Board  # noqa: E402

for (w, h, bnd, gens) in [(8192, 4096, 0, 1000), (8192, 8192, 0, 500), (8192, 4096, 1, 1000), (4096, 8192, 0, 1000)]:
    with Board(w, h, bnd) as b:
        b.seed_splitmix(11)
        b.step(2)
        b.synchronize()
        t0 = time.perf_counter()
        b.step(gens)
        b.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"env": {k: os.environ.get(k) for k in ("GOL_ILV", "GOL_COOP", "GOL_COOP_MAX_CELLS")},
                          "w": w, "h": h, "boundary": bnd, "gens": gens, "us_per_gen": round(dt / gens * 1e6, 3),
                          "ilv": b.info()["ilv"], "k": b.info()["tblock_k"]}), flush=True)
