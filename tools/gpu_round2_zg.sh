#!/bin/bash
# Round 2, call zg: coop pass with the LDS slot parity as a template constant (immediate slot offsets) and the
# raw-row exchange variant removed: coop tests, interleaved A/B against HEAD.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (256|512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_resident.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "coop_ab|400|for rep in 1 2 3; do for L in prev new; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done; done"
