#!/bin/bash
# Round 2, call zk: ragged byte boards on the cooperative pass, with the packed boards' kernels byte-identical to
# HEAD: coop / parity / resident tests, ragged timing against the byte step, config 2 A/B against HEAD.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_coop|400|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_parity.py tests/test_gpu_resident.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ragged_ab|300|python -u tools/ragged_ab.py 2" \
  "coop_4096_ab|300|bash tools/coop_4096_ab.sh 4 ab/libgol_prev.so ab/libgol_new.so"
