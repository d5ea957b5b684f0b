# GPU call script (gpurun), round 5: the torus deep pass on the bounded pass's instruction stream -- running row address
# and all row DMAs at the trip's top (wp0), and the same without the seam DMA / merge (wp0ns: WRONG boards, timing
# only) -- against the default torus and the bounded pass, at the bench window.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 300 env GOL_LIB=$PWD/build/ab/libgol_wp0.so python -u -m pytest tests/test_gpu_seam.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -15 $O/parity.log; exit 1; }
tail -1 $O/parity.log
: > $O/sweep.jsonl
for rep in 1 2 3; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_wp0.so build/ab/libgol_wp0ns.so; do
    GOL_LIB=$PWD/$L timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", \"bounded\": 0, |" >> $O/sweep.jsonl || exit 1
  done
  GOL_LIB=$PWD/gameoflifewithactors_amd/libgol_hip.so timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"libgol_hip.so\", \"bounded\": 1, |" >> $O/sweep.jsonl || exit 1
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5u/sweep.jsonl"):
    r = json.loads(l); d[(r["bounded"], r["lib"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
