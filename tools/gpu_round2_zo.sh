#!/bin/bash
# Round 2, call zo: LLVM scheduling strategies for the deep pass (iterative-ilp, max-memory-clause) against the
# default build, interleaved, 65536^2 torus K = 12 and 16.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "sched_ab|600|bash tools/ab_rep.sh gpurun_out/sched_ab_zo.log 3 '2:12,16' ab/libgol_default.so ab/libgol_iterative-ilp.so ab/libgol_max-memory-clause.so; cat gpurun_out/sched_ab_zo.log"
