#!/bin/bash
# Round 2, call x: coop pass with 16-byte LDS edge records (ds_write_b128 / ds_read_b128): coop + resident
# tests, interleaved A/B against the previous commit, block depth re-check.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (256|512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_resident.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "coop_ab|400|for rep in 1 2 3; do for L in prev new; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done; done" \
  "coop_k|300|for k in 6 10 12; do echo lib=new K=\$k; GOL_COOP_K=\$k GOL_LIB=\$PWD/ab/libgol_new.so python -u tools/small_configs.py | $SEL; done"
