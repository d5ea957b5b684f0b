"""HBM traffic per launch of the step kernel from rocprofv3 PMC passes (tools/pmc_traffic.sh output),
corrected with a calibration run of known byte counts (tools/ubench/traffic_calib.hip).

    python tools/pmc_traffic.py gpurun_out/pmc_traffic KEY M > profiles/pmc_traffic.json

MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE come from the L2's memory-side request counters;
on gfx950 FETCH_SIZE reads 1/2 of a 16-B/lane streaming read, other widths are uncalibrated.  The
calibration kernels copy exactly 1 GiB per launch at 4, 8 and 16 B/lane, so for the step kernel's
access width (4*M bytes per lane) the correction factor is 1 GiB / counter bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter):
    """{kernel name: [counter value per dispatch]} (values in KB as rocprofv3 reports them)."""
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def pick(vals, needle):
    xs = [v for k, vs in vals.items() if needle in k for v in vs]
    return sum(xs) / len(xs) if xs else None


def main():
    d, key, m = sys.argv[1], sys.argv[2], int(sys.argv[3])
    width = 4 * m
    gib = float(1 << 30)
    cf, cw = per_dispatch(os.path.join(d, "calib_fetch"), "FETCH_SIZE"), per_dispatch(os.path.join(d, "calib_write"), "WRITE_SIZE")
    calib = {}
    for w in (4, 8, 16):
        f, wr = pick(cf, f"copy_w<{w}>"), pick(cw, f"copy_w<{w}>")
        calib[w] = {"fetch_kb": f, "write_kb": wr,
                    "read_factor": gib / (f * 1024) if f else None, "write_factor": gib / (wr * 1024) if wr else None}
    bf = pick(per_dispatch(os.path.join(d, "bench_fetch"), "FETCH_SIZE"), "gol_stream_step")
    bw = pick(per_dispatch(os.path.join(d, "bench_write"), "WRITE_SIZE"), "gol_stream_step")
    rf, wf = calib[width]["read_factor"], calib[width]["write_factor"]
    read_b = bf * 1024 * rf if bf and rf else None
    write_b = bw * 1024 * wf if bw and wf else None
    out = {key: {
        "bytes_per_launch": (read_b + write_b) if read_b and write_b else None,
        "read_bytes": read_b, "write_bytes": write_b,
        "raw_fetch_kb": bf, "raw_write_kb": bw, "lane_width_bytes": width,
        "calibration": calib,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of `python3 bench.py "
                  "--no-cpu-baseline`; corrected by traffic_calib (exact 1 GiB copies at the same lane width)",
    }}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
