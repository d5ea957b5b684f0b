# GPU call script (gpurun): each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ragged_state.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_state.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_state.log; exit 1; }
tail -1 $O/pytest_state.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 tools/ragged_stream_ab.py --rounds 2 --no-bytestep > $O/ragged_stream.log 2>&1 && grep -v amdgpu $O/ragged_stream.log
timeout -k 10 300 python3 tools/small_configs.py > $O/small.log 2>&1 && grep -v amdgpu $O/small.log | grep '"w": 255\|"w": 100,'
