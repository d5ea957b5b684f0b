#!/bin/bash
# Round 2, call zh (and zi: 16 owner lanes per round against 8): single-wave pass with the byte loads batched (owner lanes rows in flight per
# round): wave-pass and parity tests, config-1 call latency against the previous build.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_wave|400|python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "c1_ab|200|for rep in 1 2; do for L in prev new; do echo lib=\$L; if [ \$L = prev ]; then GOL_LIB=\$PWD/ab/libgol_prev.so python -u tools/c1_latency.py; else python -u tools/c1_latency.py; fi; done; done"
