# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit and the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_lanes.py tests/test_gpu_ragged_state.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/lanes_ab.py --rounds 2 --boards 4096x4096x0,512x512x0,512x256x0,256x256x0,1024x2048x0,2048x1024x0,4096x1024x0,2048x4096x0,4096x8192x0,8192x2048x0,8192x8192x0,8192x4096x1 --variants coop,coopc,l5,l9,l17 > $O/lanes_ab.log 2>&1; rc=$?; echo "lanes rc=$rc"; [ $rc -eq 0 ] || exit $rc
# verdict r3 item 3: the profiled board-leg command (config 2, the cooperative pass) must exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --gens-per-step 1000 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$O/bench_c2_prof.log 2>&1; rc=$?; echo "bench_c2 under rocprofv3 rc=$rc"; grep -o '"us_per_generation[a-z_]*": [0-9.]*\|"ok": [a-z]*' $GRAFT_REPO_ROOT/$O/bench_c2_prof.log | tr '\n' ' '; echo
