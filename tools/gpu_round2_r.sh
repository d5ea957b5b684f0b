#!/bin/bash
# Round 2, call r: the cooperative pass ahead of the LDS-resident pass for packed boards: whole GPU suite, smoke,
# small-board timings with the default cut-overs.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "small_default|200|python -u tools/small_configs.py"
