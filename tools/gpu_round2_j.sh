#!/bin/bash
# Round 2, call j: static issue priority by group role (GOL_PRIO=1) against the shipped library: split sweep on
# torus and bounded 65536^2, K = 12 / 16.
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=gameoflifewithactors_amd
out=gpurun_out/prio_split.log
: > $out
for b in 0 1; do
  for sp in 0.6 0.7 0.8 0.5; do
    for lib in libgol_hip_prio.so libgol_hip.so; do
      echo "boundary=$b split=$sp lib=$lib" >> $out
      GOL_SPLIT=$sp GOL_LIB=$PWD/$L/$lib timeout -k 10 120 python tools/sweep.py --ks 12,16 --passes 12 --boundary $b 2>/dev/null | grep '^{' >> $out || exit 1
    done
  done
done
