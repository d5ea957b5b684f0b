#!/bin/bash
# Round 2, call o: per-generation sync of the coop pass -- workgroup barrier (libgol_hip.so) against neighbour-wave
# LDS counters (libgol_hip_cflags.so): parity of both, then interleaved timings.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "pytest_coop_flags|300|GOL_LIB=\$PWD/$L/libgol_hip_cflags.so python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab_sync|600|for r in 1 2; do for lib in libgol_hip.so libgol_hip_cflags.so; do echo rep=\$r lib=\$lib; GOL_LIB=\$PWD/$L/\$lib python -u tools/small_configs.py | grep -E '\"w\": (512|1024|2048|4096), \"h\": (512|1024|2048|4096)'; done; done"
