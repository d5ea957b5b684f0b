#!/bin/bash
# PMC passes for one (k, ilv) on the 65536^2 board; each counter group in its own rocprofv3 run
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass).
#   tools/pmc.sh <tag> <k> <ilv> [groups]   -> gpurun_out/pmc_<tag>/g<N>/...
# groups: subset of 1..5 (default all); GOL_LIB selects a library variant, PMC_BOUNDARY=1 a bounded board.
tag=$1; k=$2; ilv=$3; groups=${4:-"1 2 3 4 5"}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_$tag
mkdir -p $out
cmd="python3 tools/sweep.py --ilv $ilv --ks $k --passes 4 --boundary ${PMC_BOUNDARY:-0}"
G[1]="FETCH_SIZE"
G[2]="WRITE_SIZE"
G[3]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
G[4]="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G[5]="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"  # at most 4 TCC counters per pass
for i in $groups; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc ${G[$i]} --output-format csv -d $out/g$i -o run -- $cmd > $out/g$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "group $i failed rc=$rc"; tail -3 $out/g$i.log; exit $rc; fi  # nothing more on the GPU
done
