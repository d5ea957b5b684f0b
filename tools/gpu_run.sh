# GPU call script (gpurun): the current measurement call; each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3t; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{' >> $O/bench_repeat.log || exit 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline 2>/dev/null | grep '^{' >> $O/bench_repeat.log || exit 1
done
python3 -c "
import json
for l in open('$O/bench_repeat.log'):
    d=json.loads(l); print(d['config']['boundary'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['traffic'] is not None, d['config']['tblock_autotune_us_per_gen'])"
