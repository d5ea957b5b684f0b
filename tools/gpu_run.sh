# GPU call script (gpurun): the current measurement call.  Every step runs under its own time limit and the first
# failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 600 python tools/diag/ragged_fault.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log; echo "diag rc=$rc"
