#!/bin/bash
# K = 1 streaming pass: halo-free strips (default) vs halo-lane strips, all layouts, 65536^2.
out=$1; : > $out
for rep in 1 2; do
  for L in base k1halo; do
    for ilv in 1 2 4; do
      echo "rep=$rep lib=$L ilv=$ilv" >> $out
      GOL_ILV=$ilv GOL_LIB=$PWD/ab/libgol_$L.so timeout -k 10 120 python tools/sweep.py --ks 1 --passes 64 2>/dev/null | grep '^{' >> $out || exit 1
    done
  done
done
