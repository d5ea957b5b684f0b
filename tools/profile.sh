#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root).  Writes under gpurun_out/prof_<tag>/.
#   tools/profile.sh <tag> <k>
# 1. kernel trace + stats of the bench command (N = 1, no CPU baseline)
# 2. separate PMC passes: FETCH_SIZE, WRITE_SIZE (HBM bytes; MI355X_MICROARCH.md "HBM": FETCH_SIZE
#    reads 1/2 of a wide coalesced stream on gfx950 -> doubled when priced), then SQ counters.
set -e
tag=${1:-r1}; k=${2:-16}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/prof_$tag
mkdir -p $out
bench="python3 bench.py --steps 16 --warmup 2 --tblock $k --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- $bench > $out/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- $bench > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- $bench > $out/write.log 2>&1
# SQ/GRBM pass (non-fatal: counter availability differs between ROCm builds)
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/sq -o run -- $bench > $out/sq.log 2>&1 || echo "sq pass failed rc=$?"
