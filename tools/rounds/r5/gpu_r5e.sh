set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 400 env GOL_LIB=$PWD/build/ab/libgol_relay.so python -u -m pytest tests/test_gpu_lanes.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matches_oracle or narrow or block_depths" > $O/relay_tests.log 2>&1; echo "rc=$?"
grep -E "PASS|FAIL|passed|failed" $O/relay_tests.log | tail -30
