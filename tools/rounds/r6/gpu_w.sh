#!/bin/bash
# round 6 (rerun after the 32-bit clamp as r6w2): one rank's pass of the N > 1 path alone on the GPU, by cap on the waves held back for the edge bands
set -e
out=gpurun_out/r6w2
mkdir -p $out
timeout -k 10 300 python tools/strip_pass_probe.py > $out/strip_pass_probe.jsonl 2> $out/strip_pass_probe.err
