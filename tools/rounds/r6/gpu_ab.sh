#!/bin/bash
# round 6 final build (pipe code object 2adf8248b16a01af): the HBM-traffic passes keyed to it, the driver's command twice,
# and a rocprofv3 kernel trace of that command
set -e
out=gpurun_out/r6ab
mkdir -p $out
timeout -k 10 600 bash tools/pmc_traffic.sh torus 32 4 > $out/pmc_traffic.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_cmd_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/trace_bench.log 2>&1
