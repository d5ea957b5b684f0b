# GPU call script (gpurun): the current measurement call; each step under its own time limit, chained so that a failure ends the call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3w; mkdir -p $O
AB_PRE=300 timeout -k 10 500 bash tools/ab_rep.sh $O/ab_cutalign_torus.log 3 "2:12" gameoflifewithactors_amd/libgol_hip.so ab/lib_cutalign.so && grep -v amdgpu $O/ab_cutalign_torus.log | grep '^{' | cut -c1-160
AB_BOUNDARY=1 AB_PRE=300 timeout -k 10 500 bash tools/ab_rep.sh $O/ab_cutalign_bounded.log 3 "2:12" gameoflifewithactors_amd/libgol_hip.so ab/lib_cutalign.so && grep -v amdgpu $O/ab_cutalign_bounded.log | grep '^{' | cut -c1-160
