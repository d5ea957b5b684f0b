#!/bin/bash
# GPU suite, then interleaved A/B of two library builds: single-board torus, ghost-row strip, bounded.
set -e
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
bash tools/ab_rep.sh gpurun_out/split_ab_torus.log 2 "2:12,16" ab/libgol_head.so ab/libgol_new.so
bash tools/ghost_ab.sh gpurun_out/split_ab_strip.log 2 12,16 ab/libgol_head.so ab/libgol_new.so
