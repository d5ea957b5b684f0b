#!/bin/bash
# PMC passes for one (k, ilv) on the 65536^2 board; each counter group in its own rocprofv3 run
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass).
#   tools/pmc.sh <tag> <k> <ilv>      -> gpurun_out/pmc_<tag>/<group>/...
tag=$1; k=$2; ilv=$3
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_$tag
mkdir -p $out
export GOL_ILV=$ilv
cmd="python3 tools/sweep.py --ks $k --passes 4"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $out/g$i -o run -- $cmd > $out/g$i.log 2>&1 || { echo "group $i failed rc=$?"; tail -3 $out/g$i.log; }
done
