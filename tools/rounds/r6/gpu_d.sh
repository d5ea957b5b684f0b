#!/bin/bash
set -e
out=gpurun_out/r6d
mkdir -p $out
cd tools/proto
for f in 0.6 0.65 0.7; do
timeout -k 10 120 ./lib_pipe_bench 65536 65536 32 1 $f > ../../$out/lib_$f.log 2>&1
timeout -k 10 120 ./pipe_proto 65536 65536 1 "S8" 0 $f $f 1 > ../../$out/proto_$f.log 2>&1
done
