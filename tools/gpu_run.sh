# GPU call script (gpurun): each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && cat $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_torus -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_torus.log 2>&1 && grep '^{' $O/bench_torus.log | cut -c1-200
python3 tools/trace_timed.py $O/prof_torus "gol_stream_step<12, 2, false, true, false>" 20 > $O/timed_launches_torus.json && cat $O/timed_launches_torus.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bounded -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline > $O/bench_bounded.log 2>&1 && grep '^{' $O/bench_bounded.log | cut -c1-200
python3 tools/trace_timed.py $O/prof_bounded "gol_stream_step<12, 2, true, false, false>" 20 > $O/timed_launches_bounded.json && cat $O/timed_launches_bounded.json
timeout -k 10 400 python3 bench.py --board 262144 --no-cpu-baseline > $O/bench_262144.log 2>&1 && grep '^{' $O/bench_262144.log | cut -c1-300
