# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit and the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4d; mkdir -p $O
GOL_LIB=$PWD/build/ab/lib_check.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_runtime.py > $O/pytest_check.log 2>&1; rc=$?; tail -30 $O/pytest_check.log; echo "pytest(check build) rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/diag/exit_probe.sh
