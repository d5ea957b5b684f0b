# GPU call script (gpurun), round 5: the N = 2 path rehearsed on the one-GPU box (two ranks on cuda:0, gloo host-staged
# halos), self-checked against the committed w2_65536_torus checkpoint and the two-strip handle leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $O/gloo2.log 2>&1; rc=$?
grep '^{' $O/gloo2.log | cut -c1-400; exit $rc
