#!/bin/bash
# round 6: pipelined-pass knobs on the fixed poll loop -- depth, shares, poll sleep
set -e
out=gpurun_out/r6l
mkdir -p $out
cd tools/proto
for f in 0.6 0.65 0.7 0.75; do
  timeout -k 10 60 ./lib_pipe_bench_s1 65536 65536 32 2 $f > ../../$out/k32_f$f.log 2>&1
  timeout -k 10 60 ./lib_pipe_bench_s1 65536 65536 16 2 $f > ../../$out/k16_f$f.log 2>&1
done
for sl in 0 2 4; do timeout -k 10 60 ./lib_pipe_bench_s$sl 65536 65536 32 2 > ../../$out/k32_sleep$sl.log 2>&1; done
