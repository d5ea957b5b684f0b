# GPU call script (gpurun): the current measurement call; each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && cat $O/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_gloo2.log 2>&1 && grep '^{' $O/bench_gloo2.log | cut -c1-400
timeout -k 10 300 python3 tools/multi_bench.py --size 65536 --parts 1,2,4 --passes 16 --weak --tblock 12 > $O/multi_weak.log 2>&1 && grep -v amdgpu $O/multi_weak.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_torus.log 2>&1 && grep '^{' $O/bench_torus.log | cut -c1-300
