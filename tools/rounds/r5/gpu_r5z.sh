# GPU call script (gpurun), round 5: the scalar-load seam words loaded at the END of the trip (GOL_SEAM_SMEM 2, after
# the trip's row DMAs have brought the lines into L2) against loading them with each row's DMAs (1, the default):
# parity, HBM fetch bytes of both (FETCH_SIZE / WRITE_SIZE passes on the same sweep board), then timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 400 env GOL_LIB=$PWD/build/ab/libgol_smem2.so python -u -m pytest tests/test_gpu_seam.py tests/test_gpu_northstar.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -15 $O/parity.log; exit 1; }
tail -1 $O/parity.log
rm -rf gpurun_out/pmc_fetch_main gpurun_out/pmc_fetch_smem2
bash tools/pmc.sh fetch_main 12 2 "1 2" || exit 1
GOL_LIB=$PWD/build/ab/libgol_smem2.so bash tools/pmc.sh fetch_smem2 12 2 "1 2" || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_main > $O/fetch_main.json && python3 tools/pmc_summary.py gpurun_out/pmc_fetch_smem2 > $O/fetch_smem2.json
python3 -c "
import json; a=json.load(open('$O/fetch_main.json')); b=json.load(open('$O/fetch_smem2.json'))
print('main', a['FETCH_SIZE'], a['WRITE_SIZE'], a.get('avg_duration_ns')); print('smem2', b['FETCH_SIZE'], b['WRITE_SIZE'], b.get('avg_duration_ns'))"
: > $O/sweep.jsonl
for rep in 1 2 3 4; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_smem2.so; do
    GOL_LIB=$PWD/$L timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", |" >> $O/sweep.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5z/sweep.jsonl"):
    r = json.loads(l); d[(r["k"], r["lib"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
