#!/bin/bash
# Round 2, call w: (1) bounded boards at least a strip wide without column masks (12-wave workgroups at K = 12);
# (2) coop pass: zero LDS pad slots (no branch per neighbour read) and interior rows stepped before the barrier.
# Parity tests, interleaved A/B against HEAD, split sweep at K = 12, rows-per-wave sweep of the coop pass, bench.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
SEL="grep -E '\"w\": (512|2048|4096|8192), \"h\": (512|2048|4096)'"
bash tools/gpu_steps.sh \
  "pytest_bounded|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -m gpu -k 'bounded or narrow' -x -q --timeout 200 --timeout-method thread" \
  "pytest_coop|300|python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_resident.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "coop_ab|400|for rep in 1 2; do for L in head new; do echo lib=\$L; GOL_LIB=\$PWD/ab/libgol_\$L.so python -u tools/small_configs.py | $SEL; done; for r in 3 4; do echo lib=new R=\$r; GOL_COOP_R=\$r GOL_LIB=\$PWD/ab/libgol_new.so python -u tools/small_configs.py | $SEL; done; done" \
  "ab_bounded|400|AB_BOUNDARY=1 bash tools/ab_rep.sh gpurun_out/ab_bounded_w.log 2 '2:12,16' ab/libgol_head.so ab/libgol_new.so; cat gpurun_out/ab_bounded_w.log" \
  "split_bounded|300|for s in 0.6 0.65 0.7 0.75; do echo split=\$s; GOL_SPLIT=\$s python -u tools/sweep.py --ks 12 --passes 16 --boundary 1; done" \
  "bench_bounded|300|python -u bench.py --steps 20 --warmup 5 --boundary bounded --no-cpu-baseline"
