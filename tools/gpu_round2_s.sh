#!/bin/bash
# Round 2, call s: the cooperative pass on 8192-wide boards at and above 2^25 cells (ilv 4) vs streaming.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "coop_wide|400|python -u tools/coop_wide.py; GOL_ILV=4 GOL_COOP_MAX_CELLS=268435456 python -u tools/coop_wide.py; GOL_COOP=0 python -u tools/coop_wide.py"
