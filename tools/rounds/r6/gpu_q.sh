#!/bin/bash
# round 6: the N > 1 path on the pipelined pass (two ranks sharing one GPU over gloo; 65536^2 per rank, ghost-row
# strips, 32-row edge bands), the strong-scaling form, and the 262144^2 single board (config 4)
set -e
out=gpurun_out/r6q
mkdir -p $out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $out/gloo2.log 2>&1
timeout -k 10 600 python bench.py --gpus 1 --board 262144 --steps 4 --warmup 1 --no-cpu-baseline > $out/bench_262144.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_strips.py > $out/pytest.log 2>&1
