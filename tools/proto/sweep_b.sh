#!/bin/bash
# round-6 prototype: remainder geometry checks, deeper pipelines, same-box library bench
set -e
# (each step bounded; a failed check stops the script)
cd tools/proto
out=../../gpurun_out/proto_d
mkdir -p $out
timeout -k 10 120 ./pipe_proto 16000 9000 3 "" 1 0.6 0.6 1 > $out/check_16000.log 2>&1
timeout -k 10 120 ./pipe_proto 8192 16384 3 "" 1 0.6 0.6 1 > $out/check_8192.log 2>&1
timeout -k 10 200 ./pipe_proto 65536 65536 20 "" 1 0.6 0.6 1 > $out/check_65536.log 2>&1
for f in 0.55 0.6 0.65; do
  timeout -k 10 120 ./pipe_proto 65536 65536 20 "" 0 $f $f 1 > $out/sweep_65536_f${f}.log 2>&1
done
cd ../..
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $out/bench_lib.log 2>&1
