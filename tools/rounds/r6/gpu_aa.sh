#!/bin/bash
# round 6: the ghost-row pipelined kernel with the 32-bit stage-0 clamp -- parity (pipe, strips, north star), the N = 2
# rehearsal over gloo on one GPU
set -e
out=gpurun_out/r6aa
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_strips.py tests/test_gpu_northstar.py > $out/pytest.log 2>&1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $out/gloo2.log 2>&1
