# GPU call script (gpurun): cooperative-pass first-poll delay 0 vs 8 on boards of <= 2048 rows.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 400 python tools/lanes_ab.py --rounds 4 --boards 2048x2048x0,2048x2048x1,2048x1024x0,4096x1024x0,4096x2048x0,8192x1024x0,4096x4096x0 --variants coop,coopd0,coopd4 > $O/coop_d.log 2>&1; rc=$?; echo "rc=$rc"
