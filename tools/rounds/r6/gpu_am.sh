#!/bin/bash
# round 6 final device code (pipelined pass object ce04b30e6e972423), part 1: the whole GPU suite and smoke()
set -e
out=gpurun_out/r6am
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
