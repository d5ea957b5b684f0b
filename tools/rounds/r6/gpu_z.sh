#!/bin/bash
# round 6: the ghost-row pipelined kernel with the stage-0 row clamp in 32-bit scalar compares (c32) against the 64-bit
# clamp (p0), both boundaries of the comparison: the wrapping kernel
set -e
out=gpurun_out/r6z
mkdir -p $out
cd tools/proto
for rep in 1 2; do
  for v in p0 c32; do
    timeout -k 10 60 ./lib_pipe_bench_$v 65536 65536 32 1 0 0 1 >> ../../$out/wrap1_$v.log 2>&1
    timeout -k 10 60 ./lib_pipe_bench_$v 65536 65536 32 1 0 0 0 >> ../../$out/wrap0_$v.log 2>&1
  done
done
