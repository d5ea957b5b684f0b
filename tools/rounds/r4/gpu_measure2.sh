# GPU call script (gpurun): round-4 measurements on the final device code.  Each step under its own limit; a step
# that times out or crashes (rc >= 124) ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4n; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ge 124 ]; then tail -20 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
step pmc_torus 400 bash tools/pmc_traffic.sh torus 12
tail -2 $O/pmc_torus.log
step pmc_bounded 400 bash tools/pmc_traffic.sh bounded 12
tail -2 $O/pmc_bounded.log
step pmc_sq_torus 300 bash tools/pmc.sh r4_torus_k12 12 2 "3 4"
PMC_BOUNDARY=1 step pmc_sq_bounded 300 bash tools/pmc.sh r4_bounded_k12 12 2 "3 4"
for split in 0.66 0.70 0.74 0.62; do
  step split_$split 120 python tools/sweep.py --ilv 2 --ks 12 --passes 16 --pre 300 --split $split
  grep '^{' $O/split_$split.log | cut -c1-120
done
