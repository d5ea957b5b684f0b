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
step lanes_ab 300 python tools/lanes_ab.py --rounds 3
grep '^{' $O/lanes_ab.log | cut -c1-150
step bench_n1_a 300 python bench.py --gpus 1 --steps 20 --warmup 5
grep -o '"value": [0-9.]*\|"verify": {[^}]*}\|"avg_launch_us": [0-9.]*\|"value_device_events": [0-9.]*\|"first_generation_timed": [0-9]*' $O/bench_n1_a.log | tr '\n' ' '; echo
for split in 0.66 0.70 0.74 0.62 0.68 0.72; do
  step split_$split 120 python tools/sweep.py --ilv 2 --ks 12 --passes 16 --pre 300 --split $split
  grep '^{' $O/split_$split.log | cut -c1-120
done
step bench_bounded 300 python bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline
grep -o '"value": [0-9.]*\|"verify": {[^}]*}\|"avg_launch_us": [0-9.]*' $O/bench_bounded.log | tr '\n' ' '; echo
step pmc_torus 600 bash tools/pmc_traffic.sh torus 12
tail -2 $O/pmc_torus.log
step pmc_bounded 600 bash tools/pmc_traffic.sh bounded 12
tail -2 $O/pmc_bounded.log
step pmc_sq_torus 300 bash tools/pmc.sh r4_torus_k12 12 2 "3 4"
PMC_BOUNDARY=1 step pmc_sq_bounded 300 bash tools/pmc.sh r4_bounded_k12 12 2 "3 4"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify --handle-parts 0 > $GRAFT_REPO_ROOT/$O/trace_bench.log 2>&1; echo "== trace_bench rc=$?"
grep -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' $GRAFT_REPO_ROOT/$O/trace_bench.log | tr '\n' ' '; echo
