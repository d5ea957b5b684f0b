"""Per-kernel launch statistics from a rocprofv3 kernel trace, restricted to the bench's TIMED launches.

rocprofv3 --stats averages every launch of a kernel, including the bench's depth race and warmup passes.  bench.py
launches the timed passes last (before its K = 1 reference passes, a different kernel), so the timed launches of the
dominant kernel are its last `steps` dispatches in the trace.

    python tools/trace_timed.py gpurun_out/prof "gol_stream_step<12, 2, false, true, false>" 20 > timed.json
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, needle, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if needle in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    timed = rows[-n:]
    us = [(e - s) / 1e3 for s, e, _ in timed]
    out = {
        "kernel": timed[0][2] if timed else needle,
        "dispatches_in_trace": len(rows),
        "timed_dispatches": len(timed),
        "avg_us": round(statistics.mean(us), 3) if us else None,
        "min_us": round(min(us), 3) if us else None,
        "max_us": round(max(us), 3) if us else None,
        "all_dispatches_avg_us": round(statistics.mean((e - s) / 1e3 for s, e, _ in rows), 3) if rows else None,
        "source": "rocprofv3 --kernel-trace: the last `timed_dispatches` launches of the kernel (the bench's timed "
                  "region), tools/trace_timed.py",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
