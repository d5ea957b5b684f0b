#!/bin/bash
# round 6: pipelined-pass shares, same-box interleaved confirmation (two rounds)
set -e
out=gpurun_out/r6n
mkdir -p $out
cd tools/proto
for rep in 1 2; do
  for cfg in "32 0.65 0" "32 0.7 0" "32 0.75 0" "32 0.8 0" "16 0.6 0" "16 0.6 0.65" "16 0.55 0.6"; do
    set -- $cfg
    timeout -k 10 60 ./lib_pipe_bench_s1 65536 65536 $1 1 $2 $3 > ../../$out/k$1_f$2_$3_r$rep.log 2>&1
  done
done
