# GPU call script (gpurun), round 5: throttling the cooperative pass's repeated polls on wide rows, where a missed
# round costs 4 KB per wave: m4err (rows of 256 words read the error word before polling, the pre-change order) and
# sent (after a miss, one granule pair per lane until it carries the tag), parity first, then interleaved against the
# main library (new poll delays, 8192-wide boards back on the cooperative pass) and the pre-change one (olderr).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5n; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity_m4err 400 env GOL_LIB=$PWD/build/ab/libgol_m4err.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_m4err.log
step parity_sent 400 env GOL_LIB=$PWD/build/ab/libgol_sent.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_sent.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 8192x4096x0,8192x2048x0,8192x4096x1,4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0 --variants coop" gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_olderr.so build/ab/libgol_m4err.so build/ab/libgol_sent.so
python3 tools/ab_summary.py $O/ab.jsonl
echo finished
