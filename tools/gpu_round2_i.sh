#!/bin/bash
# Round 2, call i: is the bounded K = 16 regression (83k vs 93k GCUPS, same instruction counts) the age-based
# group split?  Sweep GOL_SPLIT for the current and the run-d library, bounded K = 12 / 16, torus K = 12 as
# the reference.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
: > gpurun_out/split_bounded.log
for sp in 0.5 0.6 0.72 0.85 0; do
  for lib in libgol_hip.so libgol_hip_d.so; do
    echo "split=$sp lib=$lib" >> gpurun_out/split_bounded.log
    GOL_SPLIT=$sp GOL_LIB=$PWD/$L/$lib timeout -k 10 120 python tools/sweep.py --ks 12,16 --passes 12 --boundary 1 2>/dev/null | grep '^{' >> gpurun_out/split_bounded.log || exit 1
  done
done
echo "torus" >> gpurun_out/split_bounded.log
timeout -k 10 120 python tools/sweep.py --ks 12,16 --passes 12 --boundary 0 2>/dev/null | grep '^{' >> gpurun_out/split_bounded.log
