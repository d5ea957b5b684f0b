# GPU call script (gpurun), round 5: the rows-on-lanes pass at 2048-4096 wide after the error-word change (its waves all
# publish and poll, so the change cut more there), against the cooperative pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 600 tools/lib_ab.sh $O/ab.jsonl 3 "--boards 4096x4096x0,4096x4096x1,2048x2048x0,2048x1024x0,4096x1024x0 --variants coop,l9,l5,l17,l9k6,l9k10" gameoflifewithactors_amd/libgol_hip.so || exit 1
python3 tools/ab_summary.py $O/ab.jsonl
echo finished
