#!/bin/bash
# 4 waves/SIMD (16-wave workgroups) at K = 8, M = 2 against the default K = 12 in 12-wave workgroups.
out=$1; : > $out
run() { echo "rep=$rep lib=$1 split=$2 ilv=2" >> $out; GOL_ILV=2 GOL_SPLIT=$2 GOL_LIB=$PWD/ab/libgol_$1.so timeout -k 10 120 python tools/sweep.py --ks $3 --passes 16 2>/dev/null | grep '^{' >> $out; }
for rep in 1 2; do
  run base 0.72 8,12 || exit 1
  for f in 0.5 0.6 0.7; do run w16 $f 8 || exit 1; done
done
