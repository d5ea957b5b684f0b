#!/bin/bash
# Round 2, call g: loop alignment (-falign-loops=64: every large loop starts 0 mod 64 instead of a
# placement-dependent phase) A/B on torus and bounded, interleaved with the run-d library; coop pass without
# per-generation divisions.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_coop|240|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 100 --timeout-method thread" \
  "pytest_a64|400|GOL_LIB=$PWD/$L/libgol_hip_a64.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "small_coop|200|GOL_COOP=1 python -u tools/small_configs.py" \
  "ab_torus|500|bash tools/ab_rep.sh gpurun_out/ab_torus.log 3 '2:12,16' $L/libgol_hip.so $L/libgol_hip_a64.so $L/libgol_hip_prev.so" \
  "ab_bounded|500|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded.log 3 '2:12,16' $L/libgol_hip.so $L/libgol_hip_a64.so $L/libgol_hip_d.so"
