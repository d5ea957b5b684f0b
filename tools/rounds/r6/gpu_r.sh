#!/bin/bash
# round 6: static wave priority by pipeline stage (GOL_PIPE_PRIO 0 none, 1 later half, 2 earlier half, 3 last stage),
# 4 the later half at priority 0 (alignment control), interleaved, 65536^2 K = 32
set -e
out=gpurun_out/r6r2
mkdir -p $out
cd tools/proto
for rep in 1 2 3; do
  for v in 0 1 4; do timeout -k 10 60 ./lib_pipe_bench_p$v 65536 65536 32 2 >> ../../$out/k32_prio$v.log 2>&1; done
done
