#!/bin/bash
# round 6 final device code (pipelined pass object 42b5eb4e197b1fff): HBM-traffic passes torus and bounded, the
# driver's command, and its rocprofv3 kernel trace
set -e
out=gpurun_out/r6ae
mkdir -p $out
timeout -k 10 600 bash tools/pmc_traffic.sh torus 32 4 > $out/pmc_traffic_torus.log 2>&1
timeout -k 10 600 bash tools/pmc_traffic.sh bounded 32 4 > $out/pmc_traffic_bounded.log 2>&1

timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_cmd.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/trace_bench.log 2>&1
