#!/bin/bash
# round-6 prototype: interleaved rounds at the bench window (generation 300+), splits, widths; library bench
set -e
root=$(pwd)
out=$root/gpurun_out/proto_f
mkdir -p $out
cd tools/proto
for f in 0.6 0.65; do
  timeout -k 10 200 ./pipe_proto 65536 65536 3 "" 0 $f $f 1 > $out/w65536_f${f}.log 2>&1
done
timeout -k 10 200 ./pipe_proto 63488 65536 3 "" 0 0.65 0.65 1 > $out/w63488_f0.65.log 2>&1
cd $root
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/bench_lib.log 2>&1
