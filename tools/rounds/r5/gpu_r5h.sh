# GPU call script (gpurun), round 5: XCD-aware band placement of the cooperative pass (neighbour bands on one XCD)
# against the plain order, at the first-poll delays that measured best; parity of the candidate.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity_x 400 env GOL_LIB=$PWD/build/ab/libgol_g1poslx.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_x.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0 --variants coopd0,coopd2,coopd4" build/ab/libgol_g1posl.so build/ab/libgol_g1poslx.so
step ab8 600 tools/lib_ab.sh $O/ab8.jsonl 3 "--boards 8192x4096x0,8192x2048x0 --variants coopd16,coopd24,coopd32,coopd48" build/ab/libgol_g1posl.so build/ab/libgol_g1poslx.so
python3 tools/ab_summary.py $O/ab.jsonl
python3 tools/ab_summary.py $O/ab8.jsonl
