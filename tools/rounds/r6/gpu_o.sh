#!/bin/bash
# round 6: measurement of the shipped pipelined pass (split 0.75): the driver's command three times, a kernel trace
# of it, PMC traffic (FETCH / WRITE, separate passes) and SQ counters (two groups)
set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/r6o
mkdir -p $out
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_cmd_1.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_driver_cmd_2.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_driver_cmd_3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/trace_bench.log 2>&1
python3 tools/trace_timed.py $out/trace "gol_pipe_step<4, 8, 2, true>" 20 > $out/trace_timed.json
bash tools/pmc_traffic.sh torus 32 4 > $out/pmc_traffic.log 2>&1
bash tools/pmc.sh pipe32 32 4 "3 4" > $out/pmc_sq.log 2>&1
