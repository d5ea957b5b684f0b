cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_steps.sh \
  "pytest_gpu|700|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "ab_staged|400|bash tools/ab_rep.sh gpurun_out/ab_staged.log 3 '2:12,16 1:32 4:8' gameoflifewithactors_amd/libgol_hip_unstaged.so gameoflifewithactors_amd/libgol_hip.so" \
  "bench|300|python -u bench.py --steps 20 --warmup 5 --handle-parts 4"
