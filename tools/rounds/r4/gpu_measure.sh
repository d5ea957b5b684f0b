# GPU call script (gpurun): round-4 measurements on the final device code.  Each step under its own limit; a step
# that times out or crashes (rc >= 124) ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4m; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
step bench_n1_a 400 python bench.py --gpus 1 --steps 20 --warmup 5
grep -o '"value": [0-9.]*\|"verify": {[^}]*}\|"avg_launch_us": [0-9.]*\|"value_device_events": [0-9.]*\|"first_generation_timed": [0-9]*' $O/bench_n1_a.log | tr '\n' ' '; echo
step bench_bounded 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline
grep -o '"value": [0-9.]*\|"verify": {[^}]*}\|"avg_launch_us": [0-9.]*' $O/bench_bounded.log | tr '\n' ' '; echo
step bench_c5 120 python bench.py --init rle:gosper-gun@10,10+r-pentomino@180,150 --width 256 --height 256 --boundary bounded --generations 100000 --gens-per-step 50000 --steps 1 --warmup 1
grep -o '"us_per_generation[a-z_]*": [0-9.]*\|"ok": [a-z]*' $O/bench_c5.log | tr '\n' ' '; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify --handle-parts 0 > $GRAFT_REPO_ROOT/$O/trace_bench.log 2>&1; echo "== trace_bench rc=$?"
grep -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' $GRAFT_REPO_ROOT/$O/trace_bench.log | tr '\n' ' '; echo
