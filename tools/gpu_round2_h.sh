#!/bin/bash
# Round 2, call h: round-2 kernel trace of the bench command (profiles/r2), and SQ counters of the bounded
# K = 16 pass for the current library and the run-d library (same loop bodies, 83k vs 93k GCUPS), with the
# torus K = 16 pass as the reference.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
bash tools/gpu_steps.sh \
  "prof_bench|420|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2h -o run -- python3 -u bench.py --steps 20 --warmup 5" \
  "pmc_tcur|150|bash tools/pmc.sh tcur 16 2 3" \
  "pmc_bcur|150|PMC_BOUNDARY=1 bash tools/pmc.sh bcur 16 2 3" \
  "pmc_bd|150|GOL_LIB=$PWD/$L/libgol_hip_d.so PMC_BOUNDARY=1 bash tools/pmc.sh bd 16 2 3" \
  "ab_bounded|300|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded.log 2 '2:12,16' $L/libgol_hip.so $L/libgol_hip_d.so"
