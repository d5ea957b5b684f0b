# GPU call script (gpurun): lanes-pass depth on the sizes it takes by default.  Every step runs under its own time
# limit and the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 400 python tools/lanes_ab.py --rounds 3 --boards 256x256x1,256x256x0,512x512x0,1024x1024x0,1024x2048x0,8192x2048x0,8192x4096x0 --variants coop,l5,l5k6,l5k10,l9,l9k6,l9k10 > $O/lanes_k.log 2>&1; rc=$?; echo "lanes rc=$rc"; [ $rc -eq 0 ] || exit $rc
# torus deep pass: seam-DMA placement (GOL_SEAM_SPREAD 1 = shipped, 0 / 3 / 4) interleaved at generation 300
AB_PRE=300 timeout -k 10 400 bash tools/ab_rep.sh $O/ab_spread.log 3 "2:12" gameoflifewithactors_amd/libgol_hip.so build/ab/lib_spread0.so build/ab/lib_spread3.so build/ab/lib_spread4.so; rc=$?; echo "spread rc=$rc"; [ $rc -eq 0 ] || exit $rc
# the pair split around the shipped one, interleaved
for rep in 1 2 3; do for split in 0.68 0.70 0.72; do
  timeout -k 10 120 python tools/sweep.py --ilv 2 --ks 12 --passes 16 --pre 300 --split $split | grep '^{' >> $O/split_ab.log || exit 1
done; done; echo "split done"
