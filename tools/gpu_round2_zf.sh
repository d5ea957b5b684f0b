#!/bin/bash
# Round 2, call zf: bounded edge-fill strips: the last strip no longer re-stores the 32 blocks its neighbour stores
# bounded parity tests, interleaved A/B against the previous build, whole-job bench at K = 12 and 16.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
J="grep -o '\"value\": [0-9.]*\\|\"avg_launch_us\": [0-9.]*'"
bash tools/gpu_steps.sh \
  "pytest_bounded|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_strips.py tests/test_gpu_multi.py -m gpu -k 'bounded or narrow' -x -q --timeout 200 --timeout-method thread" \
  "ab_bounded|400|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded_zf.log 2 '2:12,16' ab/libgol_prev.so ab/libgol_new.so; cat gpurun_out/ab_bounded_zf.log" \
  "job_bounded|600|for k in 12 16; do echo bounded k=\$k; python -u bench.py --boundary bounded --tblock \$k --warmup 3 --no-cpu-baseline | $J; done" \
  "bench_bounded|300|python -u bench.py --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline"
