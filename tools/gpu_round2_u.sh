#!/bin/bash
# Round 2, call u: two generations per barrier in the coop pass (libgol_hip.so) vs one (libgol_hip_rows.so):
# parity of both, interleaved timings; the 8192-wide boards at the 2^26 cut-over.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_resident.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "pytest_coop_rows|300|GOL_LIB=\$PWD/$L/libgol_hip_rows.so python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab_xh|600|for r in 1 2; do for lib in libgol_hip_rows.so libgol_hip.so; do echo rep=\$r lib=\$lib; GOL_LIB=\$PWD/$L/\$lib python -u tools/small_configs.py | grep -E '\"w\": (256|512|1024|2048|4096), \"h\": (256|512|1024|2048|4096)'; done; done" \
  "coop_wide|300|python -u tools/coop_wide.py"
