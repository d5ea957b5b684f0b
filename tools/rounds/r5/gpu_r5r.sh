# GPU call script (gpurun), round 5: the interleave-4 layout (blocks of 4 words: half the cross-lane moves and funnel
# shifts per word) at its depths against the default (12, 2), 65536^2 torus and bounded at the bench window.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5r; mkdir -p $O
: > $O/sweep.jsonl
for rep in 1 2 3; do
  for b in 0 1; do
    timeout -k 10 100 python tools/sweep.py --ilv 2 --ks 12 --passes 16 --pre 300 --boundary $b 2>/dev/null | grep '^{' | sed "s/^{/{\"bounded\": $b, /" >> $O/sweep.jsonl || exit 1
    timeout -k 10 150 python tools/sweep.py --ilv 4 --ks 8,6,4 --passes 16 --pre 300 --boundary $b 2>/dev/null | grep '^{' | sed "s/^{/{\"bounded\": $b, /" >> $O/sweep.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5r/sweep.jsonl"):
    r = json.loads(l); d[(r["bounded"], r["ilv"], r["k"])].append(r["gcups"])
for k in sorted(d): print(k, "best", max(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
