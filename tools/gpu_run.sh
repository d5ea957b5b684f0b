# GPU call script (gpurun): each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f; mkdir -p $O
AB_PRE=300 timeout -k 10 400 bash tools/ab_rep.sh $O/ab_dma16_torus.log 3 "2:12" gameoflifewithactors_amd/libgol_hip.so ab/lib_dma16.so && grep -v amdgpu $O/ab_dma16_torus.log
AB_BOUNDARY=1 AB_PRE=300 timeout -k 10 400 bash tools/ab_rep.sh $O/ab_dma16_bounded.log 3 "2:12" gameoflifewithactors_amd/libgol_hip.so ab/lib_dma16.so && grep -v amdgpu $O/ab_dma16_bounded.log
