#!/bin/bash
# Round 2, call zn: the (12, 2) SIMD-group split under the driver's bench command (fresh board, generations
# ~276-516), interleaved, two rounds.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
J="grep -o '\"value\": [0-9.]*\\|\"avg_launch_us\": [0-9.]*' | head -2"
bash tools/gpu_steps.sh \
  "split_bench|700|for rep in 1 2; do for s in 0.66 0.68 0.70 0.72 0.74; do echo split=\$s; GOL_SPLIT=\$s python -u bench.py --steps 20 --warmup 5 --tblock 12 --no-cpu-baseline | $J; done; done"
