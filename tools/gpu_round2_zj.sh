#!/bin/bash
# Round 2, call zj: ragged byte boards on the cooperative pass (whole-word scratch rows, bit-level row-end
# fix-up): coop + parity tests, ragged timing against the byte step, packed coop boards against the previous build.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (256|512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_coop|400|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_parity.py tests/test_gpu_resident.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ragged_ab|300|python -u tools/ragged_ab.py 2" \
  "coop_ab|300|for L in prev new; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done"
