#!/bin/bash
# round 6: pipelined-pass shares, second sweep
set -e
out=gpurun_out/r6m
mkdir -p $out
cd tools/proto
for f in 0.8 0.85 0.9; do timeout -k 10 60 ./lib_pipe_bench_s1 65536 65536 32 2 $f > ../../$out/k32_f$f.log 2>&1; done
timeout -k 10 60 ./lib_pipe_bench_s4 65536 65536 32 2 0.8 > ../../$out/k32_f0.8_sleep4.log 2>&1
for fs in "-1 0" "0.55 0" "0.6 0.55" "0.6 0.65" "0.55 0.6" "0.58 0.58"; do
  set -- $fs
  timeout -k 10 60 ./lib_pipe_bench_s1 65536 65536 16 2 $1 $2 > ../../$out/k16_f$1_$2.log 2>&1
done
