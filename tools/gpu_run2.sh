# GPU call script (gpurun): the bounds-checking build's suite (GOL_CHECK_BOUNDS) and the ragged size rule.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g; mkdir -p $O
GOL_LIB=$PWD/build/ab/lib_check.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_runtime.py --deselect tests/test_gpu_lanes.py --deselect tests/test_gpu_ragged_stream.py --deselect tests/test_gpu_defaults.py > $O/pytest_check.log 2>&1; rc=$?; tail -8 $O/pytest_check.log; echo "pytest(check build) rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ragged_stream_ab.py --rounds 2 --passes auto,ring,m1 --boards 10001x10001x192,16383x16383x96,8193x20000x192,65535x65535x48 > $O/ragged_ab.log 2>&1; rc=$?; cut -c1-170 $O/ragged_ab.log; echo "ragged rc=$rc"
