#!/bin/bash
# Round 2, call c: the cooperative LDS-band pass (mid-size boards) -- parity first, then timings against the
# streaming pass and over the block depth; the bench with the on-box depth race.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_coop|240|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 100 --timeout-method thread" \
  "small_coop|200|python -u tools/small_configs.py" \
  "small_stream|200|GOL_COOP=0 python -u tools/small_configs.py" \
  "small_coop_k4|200|GOL_COOP_K=4 python -u tools/small_configs.py" \
  "small_coop_k16|200|GOL_COOP_K=16 python -u tools/small_configs.py" \
  "pytest_gpu|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench|300|python -u bench.py --steps 20 --warmup 5"
