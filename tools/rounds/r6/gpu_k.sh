#!/bin/bash
# round 6: the whole GPU suite on the pipelined-pass build (as the driver runs it)
set -e
out=gpurun_out/r6k
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
