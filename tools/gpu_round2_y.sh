#!/bin/bash
# Round 2, call y: time decomposition of the coop pass (diagnostic builds, wrong results by design):
# base, 2 no LDS reads, 3 no LDS traffic, 4 no band hand-off.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (512|2048|4096)'"
bash tools/gpu_steps.sh \
  "coop_dbg|400|for rep in 1 2; do for L in prev dbg2 dbg3 dbg4; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done; done"
