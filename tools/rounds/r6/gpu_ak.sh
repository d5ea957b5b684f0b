#!/bin/bash
# round 6 final device code: SQ counters of the pipelined pass, torus and bounded (tools/pmc.sh groups 3 and 4)
set -e
timeout -k 10 600 bash tools/pmc.sh pipe32_final 32 4 "3 4"
PMC_BOUNDARY=1 timeout -k 10 600 bash tools/pmc.sh pipe32_bounded_final 32 4 "3 4"
