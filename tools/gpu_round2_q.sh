#!/bin/bash
# Round 2, call q: the cooperative pass below the LDS-resident cut-over (GOL_RESIDENT_MAX_CELLS=0) against the
# default cut-overs, interleaved.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "cut_resident|400|for r in 1 2; do echo rep=\$r default; python -u tools/small_configs.py; echo rep=\$r noresident; GOL_RESIDENT_MAX_CELLS=0 python -u tools/small_configs.py; done"
