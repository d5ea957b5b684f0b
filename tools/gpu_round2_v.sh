#!/bin/bash
# Round 2, call v: coop tests (incl. the epoch wrap), block-depth sweep of the coop pass, the whole GPU suite,
# bench (torus and bounded), kernel trace of the coop pass on config 2.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "coop_k|300|for k in 4 6 8 10 12 16; do echo k=\$k; GOL_COOP_K=\$k python -u tools/small_configs.py | grep -E '\"w\": (512|2048|4096), \"h\": (512|2048|4096)'; done" \
  "pytest_gpu|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "bench|300|python -u bench.py --steps 20 --warmup 5" \
  "bench_bounded|300|python -u bench.py --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline" \
  "prof_coop|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_coop_v -o run -- python3 tools/coop_one.py 4096 4096 1000"
