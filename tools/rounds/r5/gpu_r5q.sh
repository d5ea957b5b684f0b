# GPU call script (gpurun), round 5: the single-board torus deep pass with a running row address (GOL_AB_WRAPPTR, the
# bounded pass's walk) against the row multiply, and the bounded pass; parity of the variant on the seam tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5q; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity 600 env GOL_LIB=$PWD/build/ab/libgol_wrapptr.so python -u -m pytest tests/test_gpu_seam.py tests/test_gpu_northstar.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity.log
: > $O/sweep.jsonl
for rep in 1 2 3 4; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_wrapptr.so; do
    GOL_LIB=$PWD/$L timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", \"bounded\": 0, |" >> $O/sweep.jsonl || exit 1
  done
  GOL_LIB=$PWD/gameoflifewithactors_amd/libgol_hip.so timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"libgol_hip.so\", \"bounded\": 1, |" >> $O/sweep.jsonl || exit 1
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5q/sweep.jsonl"):
    r = json.loads(l); d[(r["bounded"], r["lib"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
