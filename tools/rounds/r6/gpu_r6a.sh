# GPU call script (gpurun), round 6 start: the headline on the round-5 final build made reproducible from rocprof --
# a kernel trace of the driver's exact bench command (timed launches via tools/trace_timed.py), then three plain runs
# of the driver's command on the same box.  Results under gpurun_out/r6a/.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r6a; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-verify --no-cpu-baseline > $R/$O/trace_bench.log 2>&1
rc=$?; echo "== trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace_bench.log; exit $rc; }
python3 tools/trace_timed.py $O/trace "gol_stream_step<12, 2, false, true" 20 > $O/trace_timed.json && cat $O/trace_timed.json
grep -o '"avg_launch_us": [0-9.]*' $O/trace_bench.log | head -1
for i in 1 2 3; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1
  rc=$?; echo "== bench $i rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_$i.log | head -1) $(grep -o '"ok": [a-z]*' $O/bench_$i.log | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
echo finished
