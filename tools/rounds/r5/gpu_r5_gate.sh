# GPU call script (gpurun), round 5 final gate part 1: the whole GPU suite, smoke, the driver's bench (N = 1 torus,
# bounded), the config-2 command (torus, bounded).  Results under gpurun_out/r5final/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${GATE_TAG:-r5final}; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/pytest.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
C2="--init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000"
step bench_c2 300 python bench.py $C2
tail -1 $O/bench_c2.log
step bench_c2_bounded 300 python bench.py $C2 --boundary bounded
tail -1 $O/bench_c2_bounded.log
step bench_n1 400 python bench.py
tail -1 $O/bench_n1.log | cut -c1-600
step bench_bounded 400 python bench.py --boundary bounded
tail -1 $O/bench_bounded.log | cut -c1-600
echo finished
