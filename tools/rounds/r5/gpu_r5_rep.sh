# GPU call script (gpurun), round 5: the driver's default bench command twice more on the final build (box spread).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5rep; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_n1_$i.log 2>&1 || exit 1
  grep '^{' $O/bench_n1_$i.log | cut -c1-200
done
echo finished
