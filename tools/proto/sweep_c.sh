#!/bin/bash
# round-6 prototype: same-box A/B of board widths, depths and splits, then the library's bench command
set -e
root=$(pwd)
out=$root/gpurun_out/proto_e
mkdir -p $out
cd tools/proto
for rep in 1 2; do
  for W in 63488 65536; do
    for f in 0.6 0.65; do
      timeout -k 10 120 ./pipe_proto $W 65536 20 "D4,S" 0 $f $f 1 > $out/ab_${W}_f${f}_r${rep}.log 2>&1
    done
  done
done
cd $root
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/bench_lib.log 2>&1
