# GPU call script (gpurun): the GPU suite on the bounds-checking build (GOL_CHECK_BOUNDS: every buffer descriptor's
# range checked against its allocation; tests/conftest.py fails a test that recorded a violation), then the ragged
# size rule interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g; mkdir -p $O
GOL_LIB=$PWD/build/ab/lib_check.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_runtime.py > $O/pytest_check.log 2>&1; rc=$?; tail -3 $O/pytest_check.log; echo "pytest(check build) rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ragged_stream_ab.py --rounds 2 --passes auto,ring,m1 --boards 10001x10001x192,16383x16383x96,8193x20000x192,65535x65535x48 > $O/ragged_ab.log 2>&1; rc=$?; echo "ragged rc=$rc"
