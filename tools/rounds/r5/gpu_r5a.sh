# GPU call script (gpurun), round 5 first call: the new safety tests (two handles from two threads, tall narrow
# packed boards, the epoch set back, the ring refresh), the coop / lanes GPU files, then fresh SQ counters of the
# config-2 passes (the 60 % wait figure was from round 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_coop.py tests/test_gpu_lanes.py tests/test_gpu_ragged_stream.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -3 $O/pytest.log
step ab 300 python tools/lanes_ab.py --rounds 2 --boards 4096x4096x0 --variants coop,l9
cat $O/ab.log
cd /tmp && export TMPDIR=/tmp
G3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
G4="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
for v in coop l9; do
  for g in 3 4; do
    eval c=\$G$g
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$v/g$g -o run -- python3 $GRAFT_REPO_ROOT/tools/lanes_ab.py --rounds 1 --boards 4096x4096x0 --variants $v > $GRAFT_REPO_ROOT/$O/pmc_${v}_g$g.log 2>&1
    rc=$?; echo "== pmc $v g$g rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $GRAFT_REPO_ROOT/$O/pmc_${v}_g$g.log; exit $rc; fi
  done
done
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py $O/pmc_coop --kernel gol_band_pass > $O/sq_coop.json && cat $O/sq_coop.json
python3 tools/pmc_summary.py $O/pmc_l9 --kernel gol_lane_pass > $O/sq_l9.json && cat $O/sq_l9.json
step stamps 300 python tools/coop_stamps.py --boards 4096x4096x0,2048x2048x0,4096x4096x1 --gens 1000
cat $O/stamps.log
