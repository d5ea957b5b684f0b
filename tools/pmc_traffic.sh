#!/bin/bash
# HBM-traffic PMC passes for one bench configuration (run on the GPU box from the repo root), each counter in its own
# rocprofv3 pass under its own time limit, then the calibrated per-launch summary merged into
#   gpurun_out/pmc_traffic/pmc_traffic.json  (copy to profiles/pmc_traffic.json)
#   tools/pmc_traffic.sh [boundary] [k] [ilv]      (default: torus 12 2; torus 32 4 = the level-pipelined pass)
set -e
boundary=${1:-torus}; k=${2:-12}; m=${3:-2}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_traffic_${boundary}_k${k}_m$m
mkdir -p $out
steps=8
bench="python3 bench.py --no-cpu-baseline --no-verify --handle-parts 0 --steps $steps --warmup 1 --tblock $k --ilv $m --boundary $boundary"
calib=tools/ubench/traffic_calib
[ -x $calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $calib tools/ubench/traffic_calib.hip
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/calib_fetch -o run -- $calib > $out/calib_fetch.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "pass failed rc=$rc: $(tail -2 $out/calib_fetch.log)"; exit $rc; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/calib_write -o run -- $calib > $out/calib_write.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "pass failed rc=$rc: $(tail -2 $out/calib_write.log)"; exit $rc; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $out/bench_fetch -o run -- $bench > $out/bench_fetch.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "pass failed rc=$rc: $(tail -2 $out/bench_fetch.log)"; exit $rc; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $out/bench_write -o run -- $bench > $out/bench_write.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "pass failed rc=$rc: $(tail -2 $out/bench_write.log)"; exit $rc; }
merge=gpurun_out/pmc_traffic/pmc_traffic.json
mkdir -p gpurun_out/pmc_traffic
[ -f $merge ] || cp profiles/pmc_traffic.json $merge
python3 tools/pmc_traffic.py $out 65536 65536 $boundary $k $m $steps $merge > $merge.new && mv $merge.new $merge
python3 -c "import json;d=json.load(open('$merge'));k=[x for x in d if '_${boundary}_k${k}_m$m' in x];print({x:d[x]['bytes_per_launch'] for x in k})"
