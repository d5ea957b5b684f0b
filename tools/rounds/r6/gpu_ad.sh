#!/bin/bash
# round 6: bounded boards default to the level-pipelined pass -- the whole GPU suite, smoke, the driver's command and
# the bounded bench on the new defaults
set -e
out=gpurun_out/r6ad
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_cmd.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded > $out/bench_bounded.log 2>&1
