# GPU call script (gpurun), round 5: the three-wave group split of the deep pass (split, split2) on the 65536^2 torus
# and bounded boards at the bench window (generation 300+): production timing, then per-role tails (GOL_STAMP build).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f; mkdir -p $O
: > $O/sweep.jsonl
for rep in 1 2; do
  for f in 0.66 0.68 0.70; do
    for f2 in 0 0.72 0.76 0.80; do
      timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --split $f --split2 $f2 2>/dev/null | grep '^{' >> $O/sweep.jsonl || exit 1
    done
  done
  for f in 0.60 0.64; do
    for f2 in 0 0.68 0.72; do
      timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 --split $f --split2 $f2 2>/dev/null | grep '^{' | sed 's/^{/{"bounded": 1, /' >> $O/sweep.jsonl || exit 1
    done
  done
done
echo "== sweep done"
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5f/sweep.jsonl"):
    r = json.loads(l)
    d[(r.get("bounded", 0), r["split"], r["split2"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "all", d[k])
PY
for args in "--split 0.70" "--split 0.70 --split2 0.76" "--split 0.68 --split2 0.76"; do
  timeout -k 10 120 env GOL_LIB=$PWD/build/ab/libgol_stamp.so python tools/tail.py --k 12 --pre 300 --boundary 0 $args 2>/dev/null | grep '^{' >> $O/tails.jsonl || exit 1
done
cat $O/tails.jsonl
