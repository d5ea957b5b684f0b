# GPU call script (gpurun), round 5: the torus deep pass on halo-lane strips (board option seam -1: 17 strips of 62 as
# on the bounded board, all DMAs at the trip's top, no seam DMA) against the seam strips and the bounded pass, at the
# bench window; split pairs for the halo-lane geometry.  3 interleaved rounds, us per (12, 2) pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5p; mkdir -p $O
: > $O/sweep.jsonl
for rep in 1 2 3; do
  for c in "0 0 0" "-1 0 0" "-1 0.60 0.72" "-1 0.64 0.72" "-1 0.66 0.76"; do set -- $c
    args="--seam $1"; [ "$2" != "0" ] && args="$args --split $2 --split2 $3"
    timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 $args 2>/dev/null | grep '^{' >> $O/sweep.jsonl || exit 1
  done
  timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 2>/dev/null | grep '^{' | sed 's/^{/{"bounded": 1, /' >> $O/sweep.jsonl || exit 1
done
echo "== sweep done"
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5p/sweep.jsonl"):
    r = json.loads(l); d[(r.get("bounded", 0), r["seam"], r["split"], r["split2"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
