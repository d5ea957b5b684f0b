#!/bin/bash
# One GPU call: parity tests, the default bench line, the rocprof kernel-trace summary of the bench
# command, and the HBM-traffic PMC passes.  Each step has its own time limit; a fault/timeout stops the
# call (tools/gpu_steps.sh).
#   tools/round_gpu.sh <tag> [traffic-key]
tag=${1:-r1}
key=${2:-65536x65536_k16}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_gpu|500|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "bench|300|python -u bench.py" \
  "prof_trace|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag/trace -o run -- python3 bench.py --no-cpu-baseline" \
  "pmc|400|bash tools/pmc_traffic.sh $key 2"
