# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit and the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -8 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/lanes_ab.py --rounds 2 --boards 4096x4096x0,4096x4096x1,2048x2048x0,8192x4096x0,256x256x1,1024x1024x0 --variants coop,l9,l5,l17,l9k6,l9d0 > $O/lanes_ab.log 2>&1; rc=$?; grep '^{' $O/lanes_ab.log | cut -c1-150; echo "lanes rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/diag/exit_probe.sh
