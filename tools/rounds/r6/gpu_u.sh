#!/bin/bash
# round 6 final gate, part 2: every BASELINE config (tools/gpu_configs.sh) and the driver's bench command twice
set -e
CFG_TAG=r6u bash tools/gpu_configs.sh
out=gpurun_out/r6u
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_cmd_$i.log 2>&1
done
