#!/bin/bash
# Round 2, call za: coop pass, batched halo poll: delay before the first poll (GOL_COOP_POLL_DELAY s_sleep
# periods of 64 clocks), against the previous commit and the no-hand-off diagnostic build.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (256|512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "coop_delay|500|for rep in 1 2; do for d in prev dbg4 0 8 16 32; do echo lib=\$d; if [ \$d = prev -o \$d = dbg4 ]; then GOL_LIB=\$PWD/ab/libgol_\$d.so python -u tools/small_configs.py | $SEL; else GOL_COOP_POLL_DELAY=\$d GOL_LIB=\$PWD/ab/libgol_new.so python -u tools/small_configs.py | $SEL; fi; done; done"
