# GPU call script (gpurun), round 5 final gate part 2: profiles of the final build -- the config-2 command's kernel
# trace and SQ counters, SQ counters of the (12, 2) deep pass on both boundaries, the HBM-traffic passes re-keyed to
# this device code, and the ragged / aligned 65535-65536 boards in one window.  Results under gpurun_out/r5prof/.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r5prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
C2="--init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_c2 -o run -- python3 $R/bench.py $C2 --no-cpu-baseline > $R/$O/trace_c2.log 2>&1
rc=$?; echo "== trace_c2 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace_c2.log; exit $rc; }
G3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
G4="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
for g in 3 4; do
  eval c=\$G$g
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/$O/pmc_c2/g$g -o run -- python3 $R/bench.py $C2 --no-cpu-baseline > $R/$O/pmc_c2_g$g.log 2>&1
  rc=$?; echo "== pmc c2 g$g rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_c2_g$g.log; exit $rc; }
done
python3 tools/pmc_summary.py $O/pmc_c2 --kernel gol_band_pass > $O/sq_c2.json && cat $O/sq_c2.json
bash tools/pmc.sh torus_k12 12 2 "3 4" || exit 1
PMC_BOUNDARY=1 bash tools/pmc.sh bounded_k12 12 2 "3 4" || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_torus_k12 > $O/sq_torus_k12.json && python3 tools/pmc_summary.py gpurun_out/pmc_bounded_k12 > $O/sq_bounded_k12.json
python3 -c "
import json; t=json.load(open('$O/sq_torus_k12.json')); b=json.load(open('$O/sq_bounded_k12.json'))
print({k: round(t[k]/b[k],3) for k in t if k in b and b[k]})"
bash tools/pmc_traffic.sh torus 12 || exit 1
bash tools/pmc_traffic.sh bounded 12 || exit 1
timeout -k 10 400 python tools/ragged_stream_ab.py --rounds 2 --boards 65535x65535x96,65536x65536x96 --boundaries 1,0 --passes auto > $O/ragged_window.log 2>&1
rc=$?; echo "== ragged_window rc=$rc"; cat $O/ragged_window.log
echo finished
