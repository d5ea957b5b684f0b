#!/bin/bash
# K = 10 at 4 waves/SIMD (16-wave workgroups, spills 108 B) and at 3 (12-wave) vs the default K = 12.
out=$1; : > $out
for rep in 1 2; do
  echo "rep=$rep default k12" >> $out
  timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit 1
  for f in 0.55 0.65; do
    echo "rep=$rep k10w16 split=$f" >> $out
    GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_k10w16.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --tblock 10 2>/dev/null | grep '^{' >> $out || exit 1
  done
  echo "rep=$rep k10w12 split=0.70" >> $out
  GOL_SPLIT=0.70 GOL_LIB=$PWD/ab/libgol_k10w12.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --tblock 10 2>/dev/null | grep '^{' >> $out || exit 1
done
