#!/bin/bash
# round 6 final device code (pipelined pass object ce04b30e6e972423), part 2: HBM-traffic passes (torus, bounded), the
# driver's command twice, the bounded bench, and a rocprofv3 kernel trace of the driver's command
set -e
out=gpurun_out/r6an
mkdir -p $out
timeout -k 10 600 bash tools/pmc_traffic.sh torus 32 4 > $out/pmc_traffic_torus.log 2>&1
timeout -k 10 600 bash tools/pmc_traffic.sh bounded 32 4 > $out/pmc_traffic_bounded.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_cmd_$i.log 2>&1
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded > $out/bench_bounded.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/trace_bench.log 2>&1
