# GPU call script (gpurun), round 5: (1) ragged bounded boards with the column mask applied only by the wave holding
# the partial block (main library) against every wave masking (x1 library, same ragged code as r5j): GPU tests, then
# interleaved timings; (2) the cooperative pass's wave-edge exchange A/B (x1: sums lane-major, x2: raw rows
# lane-major) with parity first; (3) the torus deep pass priced piece by piece against the bounded pass (VERDICT r4
# item 4): zero-fill shifts instead of rotates (tsh), no seam DMA / merge (tns), both (tshns), no seam work and all
# DMAs at the trip's top (tns0) -- those libraries compute WRONG boards and are timed only.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5k; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step ragged_tests 400 python -u -m pytest tests/test_gpu_ragged_stream.py tests/test_gpu_ragged_state.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/ragged_tests.log
: > $O/ragged_ab.jsonl
for rep in 1 2; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_x1.so; do
    GOL_LIB=$PWD/$L timeout -k 10 300 python tools/ragged_stream_ab.py --rounds 1 --boards 65535x65535x96,16383x16383x96,10001x10001x192 --boundaries 1 --passes ring,auto 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", \"abrep\": $rep, |" >> $O/ragged_ab.jsonl || exit 1
  done
done
echo "== ragged_ab done"
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5k/ragged_ab.jsonl"):
    r = json.loads(l); d[(r["w"], r["h"], r["boundary"], r["pass"], r["lib"])].append(r["us_per_gen"])
for k in sorted(d): print(k, "best", min(d[k]), "all", d[k])
PY
step parity_x1 400 env GOL_LIB=$PWD/build/ab/libgol_x1.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_x1.log
step parity_x2 400 env GOL_LIB=$PWD/build/ab/libgol_x2.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_x2.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0,8192x4096x0 --variants coop,coopk6,coopk10" gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_x1.so build/ab/libgol_x2.so
python3 tools/ab_summary.py $O/ab.jsonl
: > $O/torus.jsonl
for rep in 1 2 3; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_tsh.so build/ab/libgol_tns.so build/ab/libgol_tshns.so build/ab/libgol_tns0.so; do
    GOL_LIB=$PWD/$L timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", \"bounded\": 0, |" >> $O/torus.jsonl || exit 1
  done
  GOL_LIB=$PWD/gameoflifewithactors_amd/libgol_hip.so timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"libgol_hip.so\", \"bounded\": 1, |" >> $O/torus.jsonl || exit 1
done
echo "== torus done"
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5k/torus.jsonl"):
    r = json.loads(l); d[(r["bounded"], r["lib"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
