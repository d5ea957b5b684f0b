"""HBM traffic per launch of the step kernel from rocprofv3 PMC passes (tools/pmc_traffic.sh output), corrected
with a calibration run of known byte counts (tools/ubench/traffic_calib.hip), merged into profiles/pmc_traffic.json
under bench.py's key (width x rows per GPU, boundary, depth, interleave) with the device-code fingerprint of the
library measured -- bench.py uses an entry only for the build it was taken on.

    python tools/pmc_traffic.py gpurun_out/pmc_traffic W ROWS BOUNDARY K M STEPS [json to merge into]

MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE come from the L2's memory-side request counters; on gfx950
FETCH_SIZE reads 1/2 of a streaming read, WRITE_SIZE is exact.  The calibration kernels copy exactly 1 GiB per
launch at 4, 8 and 16 B/lane, so for the step kernel's access width (4*M bytes per lane) the correction factor is
1 GiB / counter bytes.  Only the bench's timed launches count: the last STEPS dispatches of the exact kernel.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_dispatch(d, counter):
    """{kernel name: [(dispatch id, counter value)]} (values in KB as rocprofv3 reports them)."""
    vals = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals[r["Kernel_Name"]]))
                vals[r["Kernel_Name"]][key] = vals[r["Kernel_Name"]].get(key, 0.0) + float(r["Counter_Value"])
    return {k: sorted(v.items()) for k, v in vals.items()}


def pick(vals, needle, last=0):
    xs = [x for k, vs in vals.items() if needle in k for _, x in vs]
    if last:
        xs = xs[-last:]
    return (sum(xs) / len(xs), len(xs)) if xs else (None, 0)


def main():
    d = sys.argv[1]
    W, rows, boundary, k, m, steps = sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
    merge = sys.argv[8] if len(sys.argv) > 8 else None
    from gameoflifewithactors_amd import _lib
    from bench import traffic_key

    width = 4 * m
    gib = float(1 << 30)
    cf, cw = per_dispatch(os.path.join(d, "calib_fetch"), "FETCH_SIZE"), per_dispatch(os.path.join(d, "calib_write"), "WRITE_SIZE")
    calib = {}
    for w in (4, 8, 16):
        f, _ = pick(cf, f"copy_w<{w}>")
        wr, _ = pick(cw, f"copy_w<{w}>")
        calib[w] = {"fetch_kb": f, "write_kb": wr,
                    "read_factor": gib / (f * 1024) if f else None, "write_factor": gib / (wr * 1024) if wr else None}
    if m == 4 and k in (16, 32):  # the level-pipelined pass (csrc/gol_pipe.hip): D, S, P, WRAP, BND
        name = f"gol_pipe_step<4, {k // 4}, {64 // k}, " + ("false, true>" if boundary == "bounded" else "true, false>")
    else:
        name = f"gol_stream_step<{k}, {m}, {'true' if boundary == 'bounded' else 'false'}, "
        name += "false" if boundary == "bounded" else "true"
    bf, nf = pick(per_dispatch(os.path.join(d, "bench_fetch"), "FETCH_SIZE"), name, steps)
    bw, nw = pick(per_dispatch(os.path.join(d, "bench_write"), "WRITE_SIZE"), name, steps)
    rf, wf = calib[width]["read_factor"] if width in calib else None, calib[width]["write_factor"] if width in calib else None
    read_b = bf * 1024 * rf if bf and rf else None
    write_b = bw * 1024 * wf if bw and wf else None
    alg = 2 * int(W) * int(rows) / 8
    key = traffic_key(int(W), int(rows), boundary, k, m)
    entry = {
        "bytes_per_launch": (read_b + write_b) if read_b and write_b else None,
        "read_bytes": read_b, "write_bytes": write_b,
        "traffic_over_algorithmic": ((read_b + write_b) / alg) if read_b and write_b else None,
        "raw_fetch_kb": bf, "raw_write_kb": bw, "dispatches_averaged": [nf, nw], "kernel": name,
        "lane_width_bytes": width, "calibration": calib,
        "device_code": _lib.device_code_fingerprint(kernel="gol_pipe_step" if m == 4 and k in (16, 32) else "gol_stream_step"),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of bench.py (fixed depth, no "
                  "CPU baseline), the last STEPS (timed) dispatches of the kernel; corrected by traffic_calib (exact 1 "
                  "GiB copies at the same lane width)",
    }
    out = {}
    if merge and os.path.exists(merge):
        with open(merge) as f:
            out = json.load(f)
    out[key] = entry
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
