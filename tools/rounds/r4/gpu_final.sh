# GPU call script (gpurun): the round's final build -- the GPU suite, the driver's bench line (twice), bounded, the
# board legs of configs 2 and 5 and a kernel trace of the bench (the PMC traffic keys were taken on the same device
# code, fingerprint 85b52a5008baf800: gpurun_out/r4z).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4y; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -8 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -2 $O/pytest.log
step bench_n1 400 python bench.py --gpus 1 --steps 20 --warmup 5
grep -o '"value": [0-9.]*\|"ok": [a-z]*\|"avg_launch_us": [0-9.]*' $O/bench_n1.log | tr '\n' ' '; echo
step bench_n1_2 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
grep -o '"value": [0-9.]*\|"ok": [a-z]*\|"avg_launch_us": [0-9.]*' $O/bench_n1_2.log | tr '\n' ' '; echo
step bench_bounded 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline
grep -o '"value": [0-9.]*\|"ok": [a-z]*\|"avg_launch_us": [0-9.]*' $O/bench_bounded.log | tr '\n' ' '; echo
step bench_c2 120 python bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --gens-per-step 1000 --steps 1 --warmup 1
grep -o '"us_per_generation[a-z_]*": [0-9.]*\|"ok": [a-z]*' $O/bench_c2.log | tr '\n' ' '; echo
step bench_c5 120 python bench.py --init rle:gosper-gun@10,10+r-pentomino@180,150 --width 256 --height 256 --boundary bounded --generations 100000 --gens-per-step 50000 --steps 1 --warmup 1
grep -o '"us_per_generation[a-z_]*": [0-9.]*\|"ok": [a-z]*' $O/bench_c5.log | tr '\n' ' '; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify --handle-parts 0 > $GRAFT_REPO_ROOT/$O/trace_bench.log 2>&1; echo "== trace_bench rc=$?"
grep -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' $GRAFT_REPO_ROOT/$O/trace_bench.log | tr '\n' ' '; echo
