#!/bin/bash
# Round 2, call p: SQ counters of the cooperative pass on 4096^2 and 2048^2 (2 launches of 1000 generations each).
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_coop
mkdir -p $out
for sz in 4096 2048; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $out/s$sz -o run -- python3 tools/coop_one.py $sz $sz 1000 > $out/s$sz.log 2>&1 || { echo "pmc $sz failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS --output-format csv -d $out/t$sz -o run -- python3 tools/coop_one.py $sz $sz 1000 > $out/t$sz.log 2>&1 || echo "pmc2 $sz failed"
done
echo done
