#!/bin/bash
# Parity of the GOL_ADDC_WEST build, then whole-job bench A/B against the default build (interleaved).
set -e
GOL_LIB=$PWD/ab/libgol_addc.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_strips.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/addc_parity.log 2>&1
out=gpurun_out/addc_ab.log; : > $out
for rep in 1 2 3; do
  for L in base addc; do
    echo "rep=$rep lib=$L" >> $out
    GOL_LIB=$PWD/ab/libgol_$L.so timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>/dev/null | grep '^{' >> $out
  done
done
