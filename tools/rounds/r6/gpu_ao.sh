#!/bin/bash
# round 6 final device code: the N = 2 path over gloo on one GPU (torus and bounded) and one rank's pass alone
set -e
out=gpurun_out/r6ao
mkdir -p $out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $out/gloo2_torus.log 2>&1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --boundary bounded > $out/gloo2_bounded.log 2>&1
timeout -k 10 300 python tools/strip_pass_probe.py --caps none > $out/strip_pass_probe.jsonl 2> $out/strip_pass_probe.err
