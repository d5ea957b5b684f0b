# GPU call script (gpurun), round 5: cooperative-pass variants A/B (16-byte granules, positive LDS offsets), their
# parity on the coop test file, interleaved timing at configs-2-like sizes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity_posg16 400 env GOL_LIB=$PWD/build/ab/libgol_posg16.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -2 $O/parity_posg16.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,8192x4096x0 --variants coop" build/ab/libgol_base.so build/ab/libgol_g16.so build/ab/libgol_pos.so build/ab/libgol_posg16.so
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r5b/ab.jsonl"):
    r = json.loads(l)
    if "us_per_gen" in r:
        d[(r["w"], r["h"], r["boundary"], r["lib"])].append(r["us_per_gen"])
for k in sorted(d):
    v = d[k]
    print(k, "best %.4f mean %.4f" % (min(v), sum(v) / len(v)), v)
PY
