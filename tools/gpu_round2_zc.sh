#!/bin/bash
# Round 2, call zc: bounded 65536^2 over the whole 10k-generation job at K = 12 (12-wave workgroups, no column
# masks) and K = 16, interleaved; torus K = 12 beside them.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "job_bounded|600|for rep in 1 2; do for k in 12 16; do echo bounded k=\$k; python -u bench.py --boundary bounded --tblock \$k --warmup 3 --no-cpu-baseline | grep -o '\"value\": [0-9.]*\\|\"avg_launch_us\": [0-9.]*\\|\"generations_timed\": [0-9]*'; done; done; echo torus k=12; python -u bench.py --tblock 12 --warmup 3 --no-cpu-baseline | grep -o '\"value\": [0-9.]*\\|\"avg_launch_us\": [0-9.]*\\|\"generations_timed\": [0-9]*'"
