import time, json, sys
sys.path.insert(0, '/root/repo')
from gameoflifewithactors_amd import Board
for (w, h, bnd, gens, seed) in [(100, 100, 0, 100, 'dotnet'), (4096, 4096, 0, 1000, 'dotnet'), (256, 256, 1, 100000, 'rle'), (4096, 4096, 0, 100000, 'rle')]:
    with Board(w, h, bnd) as b:
        if seed == 'dotnet':
            b.seed_dotnet(42)
        else:
            b.place_rle("b2o$2o$bo!", w // 2, h // 2)
        b.step(2); b.synchronize()
        t0 = time.perf_counter(); b.step(gens); b.synchronize(); dt = time.perf_counter() - t0
        print(json.dumps({"w": w, "h": h, "boundary": bnd, "gens": gens, "ms": round(dt * 1e3, 3), "us_per_gen": round(dt / gens * 1e6, 3), "gcups": round(w * h * gens / dt / 1e9, 2), "k": b.info()["tblock_k"]}), flush=True)
