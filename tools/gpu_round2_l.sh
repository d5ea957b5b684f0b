#!/bin/bash
# Round 2, call l: the register-band pass on by default for 2^17 < cells <= 2^25 (interleaved blocks on 4096 /
# 8192-wide boards): coop parity, the whole GPU suite, timings and the rows-per-wave knob.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "small_default|200|python -u tools/small_configs.py" \
  "small_r4|200|GOL_COOP_R=4 python -u tools/small_configs.py" \
  "small_k16r4|200|GOL_COOP_K=16 GOL_COOP_R=4 python -u tools/small_configs.py" \
  "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
