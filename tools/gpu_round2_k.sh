#!/bin/bash
# Round 2, call k: the register-band cooperative pass (gol_coop.hip rewritten): parity first, then timings at
# block depths 8 / 16 against the streaming pass.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -v --timeout 120 --timeout-method thread" \
  "small_coop8|200|GOL_COOP=1 python -u tools/small_configs.py" \
  "small_coop16|200|GOL_COOP=1 GOL_COOP_K=16 python -u tools/small_configs.py" \
  "small_coop4|200|GOL_COOP=1 GOL_COOP_K=4 python -u tools/small_configs.py" \
  "small_stream|200|GOL_COOP=0 python -u tools/small_configs.py"
