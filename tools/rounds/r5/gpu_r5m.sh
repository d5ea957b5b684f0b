# GPU call script (gpurun), round 5: first-poll delays of the cooperative pass once the error word left the hand-off's
# critical path (the first poll now goes out a memory round trip earlier): 8192-wide rows (slower at delay 24 in r5l),
# 2048^2 and 4096^2; and the rows-on-lanes pass on 8192-wide boards against the cooperative one.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5m; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step wide 600 tools/lib_ab.sh $O/wide.jsonl 3 "--boards 8192x4096x0,8192x2048x0,8192x4096x1 --variants coopd24,coopd40,coopd64,coopd96,coopd128,l9,l9d16,l9d32" gameoflifewithactors_amd/libgol_hip.so
python3 tools/ab_summary.py $O/wide.jsonl
step mid 600 tools/lib_ab.sh $O/mid.jsonl 3 "--boards 4096x4096x0,2048x2048x0,2048x1024x0,1024x1024x0 --variants coopd0,coopd2,coopd4,coopd8" gameoflifewithactors_amd/libgol_hip.so
python3 tools/ab_summary.py $O/mid.jsonl
step small 600 tools/lib_ab.sh $O/small.jsonl 3 "--boards 256x256x1,512x512x0,1024x2048x0 --variants l3,l3d0,l3d4,l3d16" gameoflifewithactors_amd/libgol_hip.so
python3 tools/ab_summary.py $O/small.jsonl
echo finished
