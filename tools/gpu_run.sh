# GPU call script (gpurun): cooperative-pass depth and poll delay at config 2's size (plain launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 400 python tools/lanes_ab.py --rounds 3 --boards 4096x4096x0,4096x4096x1,2048x2048x0 --variants coop,coopk6,coopk10,coopk12,coopd0,coopd4,coopd16,coopd32 > $O/coop_kd.log 2>&1; rc=$?; echo "coop rc=$rc"; [ $rc -eq 0 ] || exit $rc
