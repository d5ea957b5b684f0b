#!/bin/bash
# Round 2, call b: GPU suite (staged deep pass + single-wave small-board pass), the exchange variants'
# parity subset, an interleaved A/B of the exchange variants at 65536^2, the small-board timings.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_gpu|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "pytest_x1|300|GOL_LIB=$PWD/$L/libgol_hip_x1.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'packed_step or deep_pass or temporal_block or golden or light_cone'" \
  "pytest_x2|300|GOL_LIB=$PWD/$L/libgol_hip_x2.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'packed_step or deep_pass or temporal_block or golden or light_cone'" \
  "ab_xlane|500|bash tools/ab_rep.sh gpurun_out/ab_xlane.log 3 '2:12,16' $L/libgol_hip_unstaged.so $L/libgol_hip.so $L/libgol_hip_x1.so $L/libgol_hip_x2.so" \
  "small_default|200|python -u tools/small_configs.py" \
  "small_nowave|200|GOL_WAVE_RESIDENT=0 python -u tools/small_configs.py"
