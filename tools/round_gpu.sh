#!/bin/bash
# One GPU call: parity tests, the default bench line, and the rocprof kernel-trace summary of the bench
# command.  Each step has its own time limit; a fault/timeout stops the call (tools/gpu_steps.sh).
#   tools/round_gpu.sh <tag>
tag=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
exec_steps=tools/gpu_steps.sh
bash $exec_steps \
  "pytest_gpu|400|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench|300|python -u bench.py" \
  "prof_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag/trace -o run -- python3 bench.py --no-cpu-baseline"
