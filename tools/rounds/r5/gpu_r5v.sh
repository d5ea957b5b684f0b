# GPU call script (gpurun), round 5: the torus deep pass compiled without the seam geometry (GOL_AB_NOSEAM: halo-lane
# strips of 62 as on the bounded board, all row DMAs at the trip top, no seam DMA), with the row multiply (noseam) and
# with the running row address (noseamwp), against the default torus and the bounded pass; parity first.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 300 env GOL_LIB=$PWD/build/ab/libgol_noseam.so python -u -m pytest tests/test_gpu_seam.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -15 $O/parity.log; exit 1; }
tail -1 $O/parity.log
: > $O/sweep.jsonl
for rep in 1 2 3; do
  for L in gameoflifewithactors_amd/libgol_hip.so build/ab/libgol_noseam.so build/ab/libgol_noseamwp.so; do
    GOL_LIB=$PWD/$L timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", \"bounded\": 0, |" >> $O/sweep.jsonl || exit 1
  done
  GOL_LIB=$PWD/gameoflifewithactors_amd/libgol_hip.so timeout -k 10 100 python tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"libgol_hip.so\", \"bounded\": 1, |" >> $O/sweep.jsonl || exit 1
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5v/sweep.jsonl"):
    r = json.loads(l); d[(r["bounded"], r["lib"])].append(r["us_per_pass"])
for k in sorted(d): print(k, "best", min(d[k]), "mean %.1f" % (sum(d[k]) / len(d[k])), "all", d[k])
PY
echo finished
