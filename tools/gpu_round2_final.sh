#!/bin/bash
# Round 2, final evidence on HEAD: whole GPU suite, smoke(), the driver's bench command (torus, CPU baselines),
# its rocprofv3 kernel trace, the bounded bench and the small/mid-size configs.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_gpu|1000|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench|400|python -u bench.py --steps 20 --warmup 5" \
  "prof_bench|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench_final -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline" \
  "bench_bounded|300|python -u bench.py --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline" \
  "small_configs|300|python -u tools/small_configs.py"
