#!/bin/bash
# round 6: the library with the asm poll loop -- parity, north star, bench (pipe and round-5 pass), smoke
set -e
out=gpurun_out/r6j
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_defaults.py > $out/pytest_pipe.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_northstar.py > $out/pytest_northstar.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_pipe_$r.log 2>&1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --ilv 2 --tblock 12 > $out/bench_ilv2_$r.log 2>&1
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
