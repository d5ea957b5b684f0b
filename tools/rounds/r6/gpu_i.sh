#!/bin/bash
# round 6: aligned asm poll loop -- padding parity and poll-loop alignment
set -e
out=gpurun_out/r6i
mkdir -p $out
cd tools/proto
for n in p0 p1 p2 p3 a3 a4 a5; do timeout -k 10 60 ./transplant_$n 1 > ../../$out/$n.log 2>&1; done
