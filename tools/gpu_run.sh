# GPU call script (gpurun): each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ragged_stream.py tests/test_gpu_coop.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_ragged.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_ragged.log; exit 1; }
tail -1 $O/pytest_ragged.log
timeout -k 10 400 python3 tools/ragged_stream_ab.py --rounds 2 > $O/ragged_stream.log 2>&1 && grep -v amdgpu $O/ragged_stream.log
timeout -k 10 300 python3 tools/ragged_stream_ab.py --rounds 2 --boards 10001x10001x200,16383x16383x100 --ks 8,16,24,32 --no-bytestep > $O/ragged_k.log 2>&1 && grep -v amdgpu $O/ragged_k.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ragged -o run -- python3 tools/ragged_stream_ab.py --rounds 1 --boards 65535x65535x48,10001x10001x200 --boundaries 0 --no-bytestep > $O/prof_ragged.log 2>&1 && cat $O/prof_ragged/run_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --gens-per-step 1000 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c2.log 2>&1 && grep -v amdgpu $O/bench_c2.log && cat $O/prof_c2/run_kernel_stats.csv
