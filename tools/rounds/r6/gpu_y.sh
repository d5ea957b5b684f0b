#!/bin/bash
# round 6: why the ghost-row pipelined kernel is slower -- ghost rows 32 (the rank strip), 0 (clamped at the buffer's
# ends), 64, 512, against the wrapping kernel
set -e
out=gpurun_out/r6y
mkdir -p $out
cd tools/proto
for rep in 1 2; do
  timeout -k 10 60 ./lib_pipe_bench_p0 65536 65536 32 1 0 0 1 >> ../../$out/wrap1.log 2>&1
  for g in 32 0 64 512; do timeout -k 10 60 ./lib_pipe_bench_p0 65536 65536 32 1 0 0 0 $g >> ../../$out/wrap0_g$g.log 2>&1; done
done
