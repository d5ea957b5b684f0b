# GPU call script (gpurun): lanes-pass depth on the sizes it takes by default.  Every step runs under its own time
# limit and the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 400 python tools/lanes_ab.py --rounds 3 --boards 256x256x1,256x256x0,512x512x0,1024x1024x0,1024x2048x0,8192x2048x0,8192x4096x0 --variants coop,l5,l5k6,l5k10,l9,l9k6,l9k10 > $O/lanes_k.log 2>&1; rc=$?; echo "lanes rc=$rc"; [ $rc -eq 0 ] || exit $rc
