# GPU call script (gpurun): 128-column lanes windows (m = 3) against 256 (m = 5) on the narrow boards, and their tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/lanes_ab.py --rounds 3 --boards 256x256x1,256x256x0,512x512x0,1024x1024x0,1024x2048x0,512x4096x0 --variants coop,l3,l5 > $O/lanes_m3.log 2>&1; rc=$?; echo "lanes rc=$rc"; [ $rc -eq 0 ] || exit $rc
