"""Where a cooperative-pass block goes (diagnostic build GOL_COOP_STAMP=1 of csrc/gol_coop.hip, never shipped).

Per band, wave and block the build records (s_memrealtime, 10 ns) when the wave issued its hand-off stores and when its
poll for the block's halo rows returned.  From those, per band and block:
  * compute  = the band's last publisher's store time - the band's last poller's return (the block's generations);
  * wait     = the band's last poller's return - the band's own last store of the block before (publish -> go);
  * hop_top  = when the top-halo pollers had their rows - when the band above had issued its bottom rows' stores;
  * hop_bot  = the same for the bottom halo and the band below.
Prints percentiles (us) as one JSON line per board.

    python tools/coop_stamps.py [--lib build/ab/libgol_cstamp.so] [--boards 4096x4096x0,...] [--gens 1000]
(--build compiles the variant here; run the tool itself on the GPU box.)
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "build", "ab", "libgol_cstamp.so")
WAVES, BANDS, BLOCKS = 16, 256, 128


def pct(xs, ps=(10, 50, 90, 99)):
    xs = sorted(xs)
    if not xs:
        return None
    return {f"p{p}": round(xs[min(len(xs) - 1, int(len(xs) * p / 100))], 3) for p in ps}


def analyse(st, nb, nblk, K, R, B):
    """st[band][wave][blk][0 = stores issued, 1 = poll returned], 10 ns ticks; B rows in the tallest band."""
    comp, wait, hop_t, hop_b = [], [], [], []
    import numpy as np

    st = st.astype(np.int64)
    for b in range(nb):
        # waves publishing the band's top K rows (local rows [K, 2K)) and bottom K rows (local [B, B + K)), and the
        # waves polling the top halo (local [0, K)) and the bottom halo (local [K + B, 2K + B))
        for n in range(1, min(nblk, BLOCKS) - 1):
            go = st[b, :, n, 1]
            if (go == 0).any():
                continue
            G = go.max() / 100.0
            P = st[b, :, n, 0].max() / 100.0
            Pprev = st[b, :, n - 1, 0].max() / 100.0
            comp.append(P - G)
            wait.append(G - Pprev)
            up, dn = (b - 1) % nb, (b + 1) % nb
            top_w = range(0, (K + R - 1) // R)
            bot_w = range((K + B) // R, min(WAVES, (2 * K + B + R - 1) // R))
            hop_t.append(max(st[b, w, n, 1] for w in top_w) / 100.0 - st[up, :, n - 1, 0].max() / 100.0)
            hop_b.append(max(st[b, w, n, 1] for w in bot_w) / 100.0 - st[dn, :, n - 1, 0].max() / 100.0)
    return {"compute_us": pct(comp), "publish_to_go_us": pct(wait), "hop_top_us": pct(hop_t),
            "hop_bottom_us": pct(hop_b), "blocks": len(comp)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=LIB)
    p.add_argument("--build", action="store_true")
    p.add_argument("--boards", default="4096x4096x0")
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--options", default="", help="extra board options name=value,...")
    a = p.parse_args()
    if a.build:
        from gameoflifewithactors_amd import build

        build.build(lib=a.lib, defines=("GOL_COOP_STAMP=1",), force=True)
        return
    os.environ["GOL_LIB"] = a.lib
    import numpy as np

    from gameoflifewithactors_amd import INIT_DOTNET_MOD2, Board, _lib

    lib = _lib.load(a.lib)
    lib.gol_debug_coop_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    extra = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.options.split(",") if kv)
    for spec in a.boards.split(","):
        w, h, bnd = (int(x) for x in spec.split("x"))
        opts = {"coop": 1, "lanes": 0}
        opts.update(extra)
        with Board(w, h, bnd, options=opts) as bd:
            bd.seed_dotnet(42, INIT_DOTNET_MOD2)
            bd.step(a.gens)
            bd.synchronize()
            us = bd.step_timed(a.gens) / a.gens
            K = bd.get_option("coop_k") or 8
            buf = np.zeros(BANDS * WAVES * BLOCKS * 2, dtype=np.uint64)
            assert lib.gol_debug_coop_stamps(buf.ctypes.data, buf.size) == 0
        st = buf.reshape(BANDS, WAVES, BLOCKS, 2)
        nb = min(BANDS, h // K)
        B = -(-h // nb)
        R = next(r for r in (1, 2, 3, 4, 6, 8) if r >= -(-(B + 2 * K) // WAVES))
        out = {"board": spec, "us_per_gen": round(us, 4), "K": K, "R": R, "B": B}
        out.update(analyse(st, nb, -(-a.gens // K), K, R, B))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
