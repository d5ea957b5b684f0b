#!/bin/bash
set -e
out=gpurun_out/r6f
mkdir -p $out
cd tools/proto
timeout -k 10 120 ./transplant 3 > ../../$out/transplant.log 2>&1
