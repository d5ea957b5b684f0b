#!/bin/bash
# Round 2, call zd: SQ / TCC counters of the (12, 2) pass, bounded against torus, same box (why bounded K = 12
# runs 523 us per launch against 442 for the torus with the same loop instruction counts).
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
PMC_BOUNDARY=1 bash tools/pmc.sh b12 12 2 "3 4 5" && bash tools/pmc.sh t12 12 2 "3 4 5" && \
python3 tools/pmc_summary.py gpurun_out/pmc_b12 > gpurun_out/pmc_b12.json && python3 tools/pmc_summary.py gpurun_out/pmc_t12 > gpurun_out/pmc_t12.json && cat gpurun_out/pmc_b12.json gpurun_out/pmc_t12.json
