# GPU call script (gpurun), round 5 final profiles after the scalar-load seam: SQ counters of the (12, 2) deep pass on
# both boundaries, the HBM-traffic passes re-keyed to the new device code, and the torus / bounded gap at the bench
# window (3 interleaved rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5prof2; mkdir -p $O
rm -rf gpurun_out/pmc_torus_k12 gpurun_out/pmc_bounded_k12 gpurun_out/pmc_traffic_torus_k12 gpurun_out/pmc_traffic_bounded_k12
bash tools/pmc.sh torus_k12 12 2 "3 4" || exit 1
PMC_BOUNDARY=1 bash tools/pmc.sh bounded_k12 12 2 "3 4" || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_torus_k12 > $O/sq_torus_k12.json && python3 tools/pmc_summary.py gpurun_out/pmc_bounded_k12 > $O/sq_bounded_k12.json
python3 -c "
import json; t=json.load(open('$O/sq_torus_k12.json')); b=json.load(open('$O/sq_bounded_k12.json'))
print({k: round(t[k]/b[k],3) for k in t if k in b and b[k]})"
bash tools/pmc_traffic.sh torus 12 || exit 1
bash tools/pmc_traffic.sh bounded 12 || exit 1
: > $O/gap.jsonl
for rep in 1 2 3; do
  for b in 0 1; do
    timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary $b 2>/dev/null | grep '^{' | sed "s/^{/{\"bounded\": $b, /" >> $O/gap.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5prof2/gap.jsonl"):
    r = json.loads(l); d[r["bounded"]].append(r["us_per_pass"])
for k in sorted(d): print("bounded" if k else "torus", "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
