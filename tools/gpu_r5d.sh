# GPU call script (gpurun), round 5: cooperative pass with every hand-off access a buffer sc1 instruction (G16=2:
# 16-byte pairs at M >= 2, 8-byte at M = 1), pipelined polls, positive LDS offsets; parity of the candidate, A/B, stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step parity_g1pos 400 env GOL_LIB=$PWD/build/ab/libgol_g1pos.so python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/parity_g1pos.log
step ab 900 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,1024x1024x0,8192x4096x0 --variants coop" build/ab/libgol_base.so build/ab/libgol_g1pos.so build/ab/libgol_g2pos.so build/ab/libgol_g1posp.so
python3 tools/ab_summary.py $O/ab.jsonl
step stamps 300 python tools/coop_stamps.py --lib build/ab/libgol_cstamp1.so --boards 4096x4096x0,2048x2048x0 --gens 1000
cat $O/stamps.log
step tail_torus 200 env GOL_LIB=$PWD/build/ab/libgol_stamp.so python tools/tail.py --k 12 --pre 300 --boundary 0
cat $O/tail_torus.log
step tail_bounded 200 env GOL_LIB=$PWD/build/ab/libgol_stamp.so python tools/tail.py --k 12 --pre 300 --boundary 1
cat $O/tail_bounded.log
