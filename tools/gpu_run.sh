# GPU call script (gpurun): the current measurement call; each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3v; mkdir -p $O
for rep in 1 2 3; do
  for sp in 0.62 0.63 0.64 0.65 0.66; do timeout -k 10 120 python3 tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 1 --split $sp 2>/dev/null | grep '^{' >> $O/split_bounded.log || exit 1; done
  for sp in 0.68 0.69 0.70 0.71; do timeout -k 10 120 python3 tools/sweep.py --ks 12 --passes 16 --pre 300 --boundary 0 --split $sp 2>/dev/null | grep '^{' >> $O/split_torus.log || exit 1; done
done
python3 -c "
import json,collections
for f in ['$O/split_bounded.log','$O/split_torus.log']:
    d=collections.defaultdict(list)
    for l in open(f):
        r=json.loads(l); d[r['split']].append(r['gcups'])
    for k,v in sorted(d.items()): print(f[-18:], k, [round(x/1e3,1) for x in v])"
