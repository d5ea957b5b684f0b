#!/bin/bash
# Round 2, call zb: whole GPU suite on HEAD + working tree, coop A/B against the previous commit, the bench
# (torus, CPU baselines) and the rocprofv3 kernel trace of the same bench command.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (100|512|2048|4096|8192), \"h\": (100|256|512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_gpu|1000|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "coop_ab|400|for rep in 1 2; do for L in prev new; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done; done" \
  "bench|400|python -u bench.py --steps 20 --warmup 5" \
  "prof_bench|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench_zb -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
