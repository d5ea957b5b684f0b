# GPU call script (gpurun), round 5: the cooperative pass with its new defaults (16-byte granules, lean generation
# loop, first poll at once up to 4096-wide rows) and the deep pass's three-wave split -- the whole GPU suite, smoke,
# the config-2 bench command with its kernel trace and SQ counters, the headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5i; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -15 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
tail -1 $O/pytest.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
C2="--init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000"
step bench_c2 300 python bench.py $C2
tail -1 $O/bench_c2.log
step bench_c2b 300 python bench.py $C2 --boundary bounded
tail -1 $O/bench_c2b.log
step bench_n1 400 python bench.py
tail -1 $O/bench_n1.log
step bench_bounded 400 python bench.py --boundary bounded
tail -1 $O/bench_bounded.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_c2 -o run -- python3 $R/bench.py $C2 --no-cpu-baseline > $R/$O/trace_c2.log 2>&1
rc=$?; echo "== trace_c2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/$O/trace_c2.log; exit $rc; }
G3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
G4="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
for g in 3 4; do
  eval c=\$G$g
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/$O/pmc_c2/g$g -o run -- python3 $R/bench.py $C2 --no-cpu-baseline > $R/$O/pmc_c2_g$g.log 2>&1
  rc=$?; echo "== pmc c2 g$g rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $R/$O/pmc_c2_g$g.log; exit $rc; fi
done
cd $R
python3 tools/pmc_summary.py $O/pmc_c2 --kernel gol_band_pass > $O/sq_c2.json && cat $O/sq_c2.json
echo finished
