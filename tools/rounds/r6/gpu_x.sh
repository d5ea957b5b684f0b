#!/bin/bash
# round 6: the ghost-row (WRAP = false) pipelined kernel -- the N > 1 interior launch -- against the single board's, and
# its code-address sensitivity (s_nop padding 0-3 at the entry), interleaved
set -e
out=gpurun_out/r6x
mkdir -p $out
cd tools/proto
for rep in 1 2; do
  for v in p0 pad0 pad1 pad2 pad3; do
    timeout -k 10 60 ./lib_pipe_bench_$v 65536 65536 32 1 0 0 1 >> ../../$out/wrap1_$v.log 2>&1
    timeout -k 10 60 ./lib_pipe_bench_$v 65536 65536 32 1 0 0 0 >> ../../$out/wrap0_$v.log 2>&1
  done
done
