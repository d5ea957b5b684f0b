#!/bin/bash
# round 6: bounded pipelined pass with the dead-row zeroing behind branches (asm) -- whole GPU suite, smoke, bounded
# and torus benches on one box
set -e
out=gpurun_out/r6ai
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline --handle-parts 0 > $out/bench_bounded_$i.log 2>&1
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --handle-parts 0 > $out/bench_torus_$i.log 2>&1
done
