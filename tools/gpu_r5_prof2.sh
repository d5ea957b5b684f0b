# GPU call script (gpurun), round 5 final profiles after the scalar-load seam: SQ counters of the (12, 2) deep pass on
# both boundaries and the HBM-traffic passes re-keyed to the new device code, then the driver's bench with them.
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
timeout -k 10 400 python bench.py --traffic-json gpurun_out/pmc_traffic/pmc_traffic.json > $O/bench_n1.log 2>&1; rc=$?
echo "== bench_n1 rc=$rc"; grep '^{' $O/bench_n1.log | cut -c1-300
echo finished
