# GPU call script (gpurun): seam DMA placement mode 5 (every 3 levels) against the shipped mode 4, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4q; mkdir -p $O
AB_PRE=300 timeout -k 10 500 bash tools/ab_rep.sh $O/ab_spread5.log 4 "2:12" gameoflifewithactors_amd/libgol_hip.so build/ab/lib_spread5.so; rc=$?; echo "spread rc=$rc"; [ $rc -eq 0 ] || exit $rc
