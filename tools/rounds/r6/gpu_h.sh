#!/bin/bash
# round 6: instruction-alignment study of the pipelined kernel (s_nop padding before the trip loop)
set -e
out=gpurun_out/r6h
mkdir -p $out
cd tools/proto
for n in 0 1 2 3 4 5 6 7 8 12; do timeout -k 10 60 ./transplant_p$n 1 > ../../$out/pad_$n.log 2>&1; done
