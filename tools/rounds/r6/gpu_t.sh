#!/bin/bash
# round 6 final gate, part 1 (rerun as r6t2 after the ghost-row fix): the whole GPU suite and smoke() on the final build
set -e
out=gpurun_out/r6t2
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
