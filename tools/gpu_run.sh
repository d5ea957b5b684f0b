# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit and the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
# lanes pass cost decomposition: full / no hand-off / generation loops only (A/B builds, wrong boards by design)
for v in full d1 d2; do
  lib=""; [ $v != full ] && lib=$PWD/build/ab/lib_lanes_$v.so
  GOL_LIB=$lib timeout -k 10 120 python tools/lanes_ab.py --rounds 2 --boards 4096x4096x0,8192x4096x0,1024x1024x0 --variants l9,l5 > $O/decomp_$v.log 2>&1; rc=$?; echo "decomp $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $O/decomp_$v.log | cut -c1-110
done
