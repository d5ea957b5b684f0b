#!/bin/bash
# round 6: same box -- the prototype and the library's pipelined pass, the round-5 pass, and a longer warmup
set -e
out=gpurun_out/r6b
mkdir -p $out
(cd tools/proto && timeout -k 10 200 ./pipe_proto 65536 65536 2 "S8" 0 0.65 0.65 1 > ../../$out/proto.log 2>&1)
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $out/bench_pipe.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify --ilv 2 --tblock 12 > $out/bench_ilv2.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 200 --no-cpu-baseline --no-verify > $out/bench_pipe_w200.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 400 --no-cpu-baseline --no-verify --ilv 2 --tblock 12 > $out/bench_ilv2_w400.log 2>&1
(cd tools/proto && timeout -k 10 200 ./pipe_proto 65536 65536 2 "S8" 0 0.65 0.65 1 > ../../$out/proto2.log 2>&1)
