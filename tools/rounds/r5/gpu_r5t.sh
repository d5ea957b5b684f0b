# GPU call script (gpurun), round 5: the bounded deep pass with its row DMAs spread over the levels (mode 4, the torus
# placement; GOL_AB_BSPREAD) against all DMAs at the trip's top; parity of the variant on the bounded tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 600 env GOL_LIB=$PWD/build/ab/libgol_bspread.so python -u -m pytest tests/test_gpu_northstar.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -15 $O/parity.log; exit 1; }
tail -1 $O/parity.log
: > $O/sweep.jsonl
for rep in 1 2 3 4; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_bspread.so; do
    GOL_LIB=$PWD/$L timeout -k 10 100 python tools/sweep.py --ks 12,16 --passes 16 --pre 300 --boundary 1 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", |" >> $O/sweep.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5t/sweep.jsonl"):
    r = json.loads(l); d[(r["k"], r["lib"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
