#!/bin/bash
# round 6: ring/counter LDS ops in asm (no vmcnt waits): harness A/B against the prototype, then parity
set -e
out=gpurun_out/r6e
mkdir -p $out
cd tools/proto
timeout -k 10 120 ./lib_pipe_bench 65536 65536 32 2 > ../../$out/lib32.log 2>&1
timeout -k 10 120 ./pipe_proto 65536 65536 2 "S8" 0 0.65 0.65 1 > ../../$out/proto.log 2>&1
timeout -k 10 120 ./lib_pipe_bench 65536 65536 16 2 > ../../$out/lib16.log 2>&1
timeout -k 10 120 ./lib_pipe_bench 65536 65536 32 2 0.6 > ../../$out/lib32_f06.log 2>&1
timeout -k 10 120 ./lib_pipe_bench 65536 65536 32 2 0.7 > ../../$out/lib32_f07.log 2>&1
cd ../..
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipe.py > $out/pytest_pipe.log 2>&1
