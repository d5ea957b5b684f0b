#!/bin/bash
# round 6: first GPU run of the level-pipelined pass in the library -- parity, defaults, north star; bench A/B
set -e
out=gpurun_out/r6a
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipe.py -k "refuses or northstar" \
  tests/test_gpu_defaults.py > $out/pytest_pipe.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_northstar.py \
  -k "shipped_defaults and torus" > $out/pytest_northstar.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_pipe_$r.log 2>&1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --ilv 2 --tblock 12 > $out/bench_ilv2_$r.log 2>&1
done
