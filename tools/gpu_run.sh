# GPU call script (gpurun): the current measurement call; each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_n1.log; exit 1; }
tail -c 1200 $O/bench_n1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $O/bench_gloo2.log 2>&1 || { echo "gloo rc=$?"; tail -20 $O/bench_gloo2.log; exit 1; }
grep -o '"verify".*' $O/bench_gloo2.log | cut -c1-900
timeout -k 10 300 python tools/ragged_stream_ab.py --rounds 2 > $O/ragged_ab.log 2>&1 || { echo "ragged rc=$?"; tail -5 $O/ragged_ab.log; exit 1; }
cut -c1-200 $O/ragged_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --gens-per-step 1000 --steps 5 > $GRAFT_REPO_ROOT/$O/bench_c2.log 2>&1; echo "c2 profiled rc=$?"
tail -c 1200 $GRAFT_REPO_ROOT/$O/bench_c2.log
