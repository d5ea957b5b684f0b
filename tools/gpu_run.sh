# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit and the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4e; mkdir -p $O
GOL_LIB=$PWD/build/ab/lib_check.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_runtime.py --deselect tests/test_gpu_lanes.py > $O/pytest_check.log 2>&1; rc=$?; tail -8 $O/pytest_check.log; echo "pytest(check build) rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -8 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/diag/exit_probe.sh
timeout -k 10 500 python tools/ragged_stream_ab.py --rounds 2 --ks 0,16 --boards 10001x10001x192,65535x65535x48,65536x65535x48 > $O/ragged_ab.log 2>&1; rc=$?; cut -c1-170 $O/ragged_ab.log; echo "ragged rc=$rc"
