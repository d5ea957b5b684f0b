# GPU call script (gpurun): pair split of the ragged bounded block rows (65535^2).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 500 python tools/ragged_split.py --rounds 2 > $O/ragged_split.log 2>&1; rc=$?; cat $O/ragged_split.log | cut -c1-120; echo "rc=$rc"
