"""Launch-tail diagnostic (needs a GOL_STAMP=1 build via GOL_LIB): one pass over a board, then the
per-wave start/end stamps (s_memrealtime, 100 MHz) -> how long the launch's waves are busy vs the
launch span.

    GOL_LIB=ab/libgol_stamp.so python tools/tail.py [--size 65536] [--k 16]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=65536)
    p.add_argument("--k", type=int, default=16)
    p.add_argument("--boundary", type=int, default=0)
    p.add_argument("--pre", type=int, default=0, help="generations stepped before the stamped passes")
    p.add_argument("--split", type=float, default=None, help="board option 'split' (fraction)")
    p.add_argument("--split2", type=float, default=None, help="board option 'split2' (fraction)")
    a = p.parse_args()
    from gameoflifewithactors_amd import Board, _lib

    lib = _lib.load()
    fn = lib.gol_debug_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_longlong]
    n = a.size
    opts = {}
    if a.split is not None:
        opts["split"] = int(a.split * 65536)
    if a.split2 is not None:
        opts["split2"] = int(a.split2 * 65536)
    with Board(n, n, a.boundary, tblock_k=a.k, options=opts) as b:
        b.seed_splitmix(1)
        if a.pre:
            b.step(a.pre)
        for rep in range(3):
            b.step(a.k)
            b.synchronize()
            buf = np.zeros(2 * 65536, np.uint64)
            fn(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), buf.size)
            t0, t1 = buf[:65536], buf[65536:]
            m = t0 > 0
            t0, t1 = t0[m].astype(np.float64) / 100.0, t1[m].astype(np.float64) / 100.0  # us
            span = t1.max() - t0.min()
            busy = t1 - t0
            ends = t1 - t0.min()
            wpb = 12 if a.k == 12 else 8
            ids = np.nonzero(m)[0]
            role_end = [round(float(np.median(ends[((ids % wpb) >> 2) == r])), 1) for r in range(wpb // 4)]
            print(json.dumps({"rep": rep, "split": a.split, "split2": a.split2, "role_end_p50_us": role_end,
                              "waves": int(m.sum()), "span_us": round(span, 1),
                              "busy_mean_us": round(busy.mean(), 1), "busy_min_us": round(busy.min(), 1),
                              "busy_max_us": round(busy.max(), 1),
                              "start_spread_us": round(t0.max() - t0.min(), 1),
                              "end_p10_us": round(float(np.percentile(ends, 10)), 1),
                              "end_p50_us": round(float(np.percentile(ends, 50)), 1),
                              "end_p90_us": round(float(np.percentile(ends, 90)), 1),
                              "util": round(busy.sum() / (span * m.sum()), 4)}), flush=True)
            if rep == 0:
                np.save(os.path.join(ROOT, "gpurun_out", f"stamps_{n}_k{a.k}_b{a.boundary}.npy"), buf)
            buf[:] = 0


if __name__ == "__main__":
    main()
