#!/bin/bash
# HBM-traffic PMC passes for the bench configuration (run on the GPU box from the repo root).
# One counter per rocprofv3 pass (FETCH_SIZE and WRITE_SIZE cannot share one), each under its own
# time limit; then the calibrated per-launch summary -> gpurun_out/pmc_traffic/pmc_traffic.json.
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_traffic
mkdir -p $out
bench="python3 bench.py --no-cpu-baseline --steps 8 --warmup 1"
calib=tools/ubench/traffic_calib
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/calib_fetch -o run -- $calib > $out/calib_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/calib_write -o run -- $calib > $out/calib_write.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/bench_fetch -o run -- $bench > $out/bench_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/bench_write -o run -- $bench > $out/bench_write.log 2>&1
python3 tools/pmc_traffic.py $out ${1:-65536x65536_k12} ${2:-2} > $out/pmc_traffic.json
cat $out/pmc_traffic.json
