#!/bin/bash
# Round 2, call d: bounded boards with edge-fill strips and masked edge trips only; 32-bit loop row
# arithmetic; parity first, then an interleaved A/B (previous kernel vs new, 8- and 12-wave bounded) on the
# bounded and torus 65536^2 boards.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_parity|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "pytest_bw12|300|GOL_LIB=$PWD/$L/libgol_hip_bw12.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'bounded or packed_step or deep_pass or golden'" \
  "ab_bounded|400|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded.log 3 '2:12,16' $L/libgol_hip_prev.so $L/libgol_hip.so $L/libgol_hip_bw12.so" \
  "ab_torus|300|bash tools/ab_rep.sh gpurun_out/ab_torus.log 3 '2:12,16' $L/libgol_hip_prev.so $L/libgol_hip.so" \
  "pytest_gpu|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
