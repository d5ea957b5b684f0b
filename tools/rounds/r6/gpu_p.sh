#!/bin/bash
# round 6: does the cooperative pass (config 2) follow its code address too?  s_nop padding at its entry, 4 builds
set -e
out=gpurun_out/r6p
mkdir -p $out
bash tools/lib_ab.sh $out/coop_pad_ab.jsonl 2 "--boards 4096x4096x0,4096x4096x1,2048x2048x0 --variants coop" \
  build/ab/libgol_coop_pad0.so build/ab/libgol_coop_pad1.so build/ab/libgol_coop_pad2.so build/ab/libgol_coop_pad3.so
