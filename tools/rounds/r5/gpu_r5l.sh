# GPU call script (gpurun), round 5: the persistent passes' error word read only while a wave waits (not before every
# hand-off poll): parity of the coop / lanes / concurrency GPU tests on the new library, then interleaved timings
# against the previous one (olderr) on the cooperative and rows-on-lanes boards.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5l; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity 600 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_lanes.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0,8192x4096x0 --variants coop" gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_olderr.so
python3 tools/ab_summary.py $O/ab.jsonl
step ab_lanes 600 tools/lib_ab.sh $O/ab_lanes.jsonl 3 "--boards 256x256x1,512x512x0,1024x1024x0,8192x2048x0,8192x4096x0 --variants l9,l5" gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_olderr.so
python3 tools/ab_summary.py $O/ab_lanes.jsonl
C2="--init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000"
step bench_c2 300 python bench.py $C2
tail -1 $O/bench_c2.log
echo finished
