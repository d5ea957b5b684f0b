# GPU call script (gpurun), round 5: the torus (12, 2) split pair re-checked on the scalar-load seam build, 4 interleaved
# rounds at the bench window.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s2; mkdir -p $O
: > $O/sweep.jsonl
for rep in 1 2 3 4; do
  for c in "0.66 0.76" "0.64 0.76" "0.68 0.76" "0.66 0.72" "0.66 0.80" "0.68 0.72"; do set -- $c
    timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --split $1 --split2 $2 2>/dev/null | grep '^{' >> $O/sweep.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5s2/sweep.jsonl"):
    r = json.loads(l); d[(r["split"], r["split2"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
