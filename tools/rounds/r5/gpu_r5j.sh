# GPU call script (gpurun), round 5: (1) ragged bounded boards on the (12, 2) kernel without its spill (VERDICT r4
# item 5): the ragged GPU tests, then 65535^2 / 16383^2 / 10001^2 per pass; (2) the cooperative pass's wave-edge
# exchange A/B: sums in planes (base), sums lane-major with ds_*_b64 (x1), raw rows lane-major (x2) -- parity of each
# variant library on the coop tests, then interleaved timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5j; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step ragged_tests 400 python -u -m pytest tests/test_gpu_ragged_stream.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/ragged_tests.log
step ragged_ab 500 python tools/ragged_stream_ab.py --rounds 2 --boards 65535x65535x48,16383x16383x96,10001x10001x192 --boundaries 1,0 --passes auto,ring,m1
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5j/ragged_ab.log"):
    if l.startswith("{"):
        r = json.loads(l); d[(r["w"], r["h"], r["boundary"], r["pass"])].append(r["us_per_gen"])
for k in sorted(d): print(k, "best", min(d[k]), "all", d[k])
PY
step parity_x1 400 env GOL_LIB=$PWD/build/ab/libgol_x1.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_x1.log
step parity_x2 400 env GOL_LIB=$PWD/build/ab/libgol_x2.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_x2.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0,8192x4096x0 --variants coop" gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_x1.so build/ab/libgol_x2.so
python3 tools/ab_summary.py $O/ab.jsonl
echo finished
