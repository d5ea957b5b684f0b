#!/bin/bash
# Round 2, call zl: coop hand-off polling, sentinel then batch (one granule per lane polled alone, then all of
# them at once) against the shipped polling: coop tests on the variant, interleaved A/B (delay 8 and 0).
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_sent|300|GOL_LIB=\$PWD/ab/libgol_sent.so python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "sent_ab|500|for rep in 1 2 3; do for L in prev sent sent0; do echo lib=\$L; if [ \$L = sent0 ]; then GOL_COOP_POLL_DELAY=0 GOL_LIB=\$PWD/ab/libgol_sent.so python -u tools/small_configs.py | $SEL; else GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; fi; done; done"
