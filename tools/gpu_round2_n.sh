#!/bin/bash
# Round 2, call n: granule hand-off (data-tagged 8-byte sc1 stores polled by the consumer lanes) in the coop
# pass: parity, then timings interleaved with the committed pass (libgol_hip_cprev.so).
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab_coop|600|for r in 1 2; do for lib in libgol_hip_cprev.so libgol_hip.so; do echo rep=\$r lib=\$lib; GOL_LIB=\$PWD/$L/\$lib python -u tools/small_configs.py | grep -E '\"w\": (512|1024|2048|4096), \"h\": (512|1024|2048|4096)'; done; done" \
  "coop_k|300|for k in 4 8 16; do echo k=\$k; GOL_COOP_K=\$k python -u tools/small_configs.py | grep -E '\"w\": (1024|2048|4096), \"h\": (1024|2048|4096)'; done"
