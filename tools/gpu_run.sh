# GPU call script (gpurun): the automatic first-poll delay -- cooperative tests and an A/B against the fixed delay 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_ragged_state.py tests/test_gpu_northstar.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/lanes_ab.py --rounds 3 --boards 2048x2048x0,2048x1024x0,4096x4096x0,4096x2048x0 --variants coop,coopd8 > $O/coop_auto.log 2>&1; rc=$?; echo "rc=$rc"
