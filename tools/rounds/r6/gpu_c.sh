#!/bin/bash
# round 6: the library's pipelined kernel in a standalone harness against the prototype, same box
set -e
out=gpurun_out/r6c
mkdir -p $out
cd tools/proto
timeout -k 10 120 ./pipe_proto 65536 65536 2 "S8" 0 0.65 0.65 1 > ../../$out/proto.log 2>&1
timeout -k 10 120 ./lib_pipe_bench 65536 65536 32 2 > ../../$out/lib.log 2>&1
timeout -k 10 120 ./lib_pipe_bench 65536 65536 16 2 > ../../$out/lib16.log 2>&1
timeout -k 10 120 ./pipe_proto 65536 65536 2 "S8" 0 0.65 0.65 1 > ../../$out/proto2.log 2>&1
