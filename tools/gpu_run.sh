# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit; a step that
# times out, aborts or crashes (rc 124 / 134 / 137 / 139 / > 128) ends the call, an ordinary failure (a failed test,
# a verify mismatch: rc 1-3) is reported and the next step runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4b; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
step bench_n1 300 python bench.py --gpus 1 --steps 20 --warmup 5
grep -o '"value": [0-9.]*\|"verify".*' $O/bench_n1.log | cut -c1-700
AB_PRE=300 step ab_seam1 500 bash tools/ab_rep.sh $O/ab_seam1_torus.log 3 "2:12 2:16" gameoflifewithactors_amd/libgol_hip.so build/ab/lib_seam0.so
grep -v amdgpu $O/ab_seam1_torus.log | cut -c1-150
step pytest 800 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
tail -15 $O/pytest.log
step bench_gloo2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2
grep -o '"value": [0-9.]*\|"verify".*' $O/bench_gloo2.log | cut -c1-900
step ragged_ab 400 python tools/ragged_stream_ab.py --rounds 2
cut -c1-170 $O/ragged_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --gens-per-step 1000 --steps 5 > $GRAFT_REPO_ROOT/$O/bench_c2.log 2>&1; echo "== c2 profiled rc=$?"
tail -c 900 $GRAFT_REPO_ROOT/$O/bench_c2.log
