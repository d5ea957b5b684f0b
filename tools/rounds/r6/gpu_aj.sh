#!/bin/bash
# round 6: smoke() with the level-pipelined pass on both boundaries
set -e
out=gpurun_out/r6aj
mkdir -p $out
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
