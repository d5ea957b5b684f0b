#!/bin/bash
# Round 2, call e: torus instruction streams restored beside the bounded edge-fill kernel; A/B against the
# previous library on torus and bounded boards; full GPU suite; bench.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_parity|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "ab_torus|400|bash tools/ab_rep.sh gpurun_out/ab_torus.log 4 '2:12,16' $L/libgol_hip_prev.so $L/libgol_hip.so" \
  "ab_bounded|400|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded.log 2 '2:12,16' $L/libgol_hip.so $L/libgol_hip_bw12.so" \
  "pytest_gpu|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench|300|python -u bench.py --steps 20 --warmup 5" \
  "bench_bounded|300|python -u bench.py --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline"
