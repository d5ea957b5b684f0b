#!/bin/bash
# round 6: stage order by age (GOL_PIPE_MAP 1: the last stage the oldest wave), interleaved with the shipped order
set -e
out=gpurun_out/r6s
mkdir -p $out
cd tools/proto
for rep in 1 2 3; do
  for v in p0 m1; do timeout -k 10 60 ./lib_pipe_bench_$v 65536 65536 32 2 >> ../../$out/k32_$v.log 2>&1; done
done
