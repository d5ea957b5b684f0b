#!/bin/bash
# Round 2, call f: the coop pass rewritten (band resident in LDS, write-through edge hand-off) and the
# single-wave pass's ballot loads: parity first, then timings; bounded A/B (previous / run-d / current
# libraries, interleaved), with the torus board before and after as a drift check.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_coop|240|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_resident.py -m gpu -x -q --timeout 100 --timeout-method thread" \
  "small_coop|200|GOL_COOP=1 python -u tools/small_configs.py" \
  "small_coop16|200|GOL_COOP=1 GOL_COOP_K=16 python -u tools/small_configs.py" \
  "ab_torus1|200|bash tools/ab_rep.sh gpurun_out/ab_torus1.log 1 '2:16' $L/libgol_hip_prev.so $L/libgol_hip.so" \
  "ab_bounded|500|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded.log 3 '2:12,16' $L/libgol_hip_prev.so $L/libgol_hip_d.so $L/libgol_hip.so" \
  "ab_torus2|200|bash tools/ab_rep.sh gpurun_out/ab_torus2.log 1 '2:16' $L/libgol_hip_prev.so $L/libgol_hip.so"
