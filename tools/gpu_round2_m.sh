#!/bin/bash
# Round 2, call m: coop pass with its own row sums before the barrier and 8-byte hand-off accesses: parity,
# then an interleaved A/B against the previous commit's pass.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab_coop|600|for r in 1 2; do for lib in libgol_hip_cprev.so libgol_hip.so; do echo rep=\$r lib=\$lib; GOL_LIB=\$PWD/$L/\$lib python -u tools/small_configs.py | grep -E '\"w\": (512|1024|2048|4096), \"h\": (512|1024|2048|4096)'; done; done"
