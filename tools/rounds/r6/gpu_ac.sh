#!/bin/bash
# round 6: bounded boards on the level-pipelined pass -- parity (pipe tests), then the pass's speed on the bounded
# 65536^2 board against the streaming pass (the bounded default), same box
set -e
out=gpurun_out/r6ac
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipe.py > $out/pytest_pipe.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline --handle-parts 0 > $out/bench_bounded_default_$i.log 2>&1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --ilv 4 --tblock 32 --no-cpu-baseline --handle-parts 0 > $out/bench_bounded_pipe_$i.log 2>&1
done
