# GPU call script (gpurun), round 5: the cooperative timeout test on every hand-off form (M = 1, 2, 4).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_coop.py -x -v -k "timeout" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/timeout.log 2>&1; rc=$?
tail -8 $O/timeout.log; exit $rc
