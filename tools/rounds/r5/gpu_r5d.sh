# GPU call script (gpurun), round 5: coop hand-off variants (16-byte global/buffer sc1 granules, positive LDS offsets,
# lean generation loop, pipelined polls) and the lanes LDS-relay hand-off: parity of the candidates, interleaved A/B,
# stamps; per-wave tails of the deep pass, torus vs bounded.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity_relay_all 400 env GOL_LIB=$PWD/build/ab/libgol_relay.so python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_relay_all.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0,8192x4096x0 --variants coop" build/ab/libgol_base.so build/ab/libgol_g1pos.so build/ab/libgol_g2pos.so build/ab/libgol_g1posp.so build/ab/libgol_g1posl.so
python3 tools/ab_summary.py $O/ab.jsonl
step ab_lanes 900 tools/lib_ab.sh $O/ab_lanes.jsonl 3 "--boards 256x256x1,256x256x0,512x512x0,1024x2048x0,8192x2048x0,4096x4096x0 --variants l3k10,l9" build/ab/libgol_base.so build/ab/libgol_relay.so
python3 tools/ab_summary.py $O/ab_lanes.jsonl
step stamps 300 python tools/coop_stamps.py --lib build/ab/libgol_cstamp1.so --boards 4096x4096x0,2048x2048x0 --gens 1000
cat $O/stamps.log
step tail_torus 200 env GOL_LIB=$PWD/build/ab/libgol_stamp.so python tools/tail.py --k 12 --pre 300 --boundary 0
cat $O/tail_torus.log
step tail_bounded 200 env GOL_LIB=$PWD/build/ab/libgol_stamp.so python tools/tail.py --k 12 --pre 300 --boundary 1
cat $O/tail_bounded.log
