#!/bin/bash
# Round 2, call zm: coop halo hand-off staged through LDS by the whole workgroup (every thread polls a share of
# the 2K halo rows, one barrier, then the halo waves copy theirs) against the shipped per-wave polling.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_stage|300|GOL_LIB=\$PWD/ab/libgol_stage.so python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "stage_ab|500|for rep in 1 2 3; do for L in prev stage; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done; done"
