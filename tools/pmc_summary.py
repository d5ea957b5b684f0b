"""Summarise rocprofv3 PMC CSVs (tools/pmc.sh output) for the step kernel: per-dispatch averages.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> [--kernel gol_stream_step]
FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived); on gfx950 FETCH_SIZE reports half of a wide
coalesced streaming read (MI355X_MICROARCH.md "HBM"), so `hbm_read_bytes` doubles it.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "gol_stream_step"
    vals = defaultdict(list)
    durs = []
    for f in glob.glob(os.path.join(d, "g*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "g*", "run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    if durs:
        out["avg_duration_ns"] = sum(durs) / len(durs)
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in out and durs:
        out["clock_ghz_est"] = out["GRBM_GUI_ACTIVE"] / 8 / (sum(durs) / len(durs))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
