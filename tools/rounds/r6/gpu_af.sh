#!/bin/bash
# round 6 (rerun as r6al): bounded pass with the dead-row test in 32-bit scalars (no 64-bit sentinel compare) --
# then the bounded bench against the torus, same box
set -e
out=gpurun_out/r6al
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_strips.py > $out/pytest_pipe.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline --handle-parts 0 > $out/bench_bounded_$i.log 2>&1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --handle-parts 0 > $out/bench_torus_$i.log 2>&1
done
