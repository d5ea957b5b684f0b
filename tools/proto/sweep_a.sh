#!/bin/bash
# round-6 prototype sweep: correctness with split + rotation, then split x rotation at 63488 x 65536
set -e
cd tools/proto
out=../../gpurun_out/proto_c
mkdir -p $out
timeout -k 10 120 ./pipe_proto 8192 4100 3 "" 1 0.6 0.6 1 > $out/check_small.log 2>&1
timeout -k 10 120 ./pipe_proto 65536 65536 3 "M4,D3" 1 0.6 0.6 1 > $out/check_65536.log 2>&1
for rot in 0 1; do
  for f in 0 0.55 0.6 0.65 0.7; do
    timeout -k 10 120 ./pipe_proto 63488 65536 20 "" 0 $f $f $rot > $out/sweep_rot${rot}_f${f}.log 2>&1
  done
done
