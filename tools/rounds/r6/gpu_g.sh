#!/bin/bash
set -e
out=gpurun_out/r6g
mkdir -p $out
cd tools/proto
for v in 0 1 2; do timeout -k 10 120 ./transplant_v$v 2 > ../../$out/transplant_v$v.log 2>&1; done
