# GPU call script (gpurun), round 5: cooperative pass (16-byte granules + lean loop) with one or two poll rounds in
# flight and first-poll delays; the deep pass's three-wave split (split, split2) confirmed over 4 interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5g; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity_p 400 env GOL_LIB=$PWD/build/ab/libgol_g1poslp.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_p.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0,8192x4096x0 --variants coop,coopd0,coopd16,coopd24" build/ab/libgol_g1posl.so build/ab/libgol_g1poslp.so
python3 tools/ab_summary.py $O/ab.jsonl
: > $O/sweep.jsonl
for rep in 1 2 3 4; do
  for c in "0.70 0" "0.66 0.76" "0.68 0.72" "0.66 0.72"; do set -- $c
    timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --split $1 --split2 $2 2>/dev/null | grep '^{' >> $O/sweep.jsonl || exit 1
  done
  for c in "0.64 0" "0.60 0.72" "0.62 0.72" "0.60 0.76"; do set -- $c
    timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 --split $1 --split2 $2 2>/dev/null | grep '^{' | sed 's/^{/{"bounded": 1, /' >> $O/sweep.jsonl || exit 1
  done
done
echo "== sweep done"
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5g/sweep.jsonl"):
    r = json.loads(l)
    d[(r.get("bounded", 0), r["split"], r["split2"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
