#!/bin/bash
out=$1; : > $out
for rep in 1 2; do
  for f in 0.6; do echo "rep=$rep lib=base split=$f ilv=1" >> $out; GOL_ILV=1 GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_base.so timeout -k 10 120 python tools/sweep.py --ks 24,32 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
  for f in 0.6 0.7; do echo "rep=$rep lib=w12all split=$f ilv=1" >> $out; GOL_ILV=1 GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_w12all.so timeout -k 10 120 python tools/sweep.py --ks 24 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
  for f in 0.55; do echo "rep=$rep lib=base split=$f ilv=4" >> $out; GOL_ILV=4 GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_base.so timeout -k 10 120 python tools/sweep.py --ks 4,8 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
  for f in 0.6 0.7; do echo "rep=$rep lib=w12all split=$f ilv=4" >> $out; GOL_ILV=4 GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_w12all.so timeout -k 10 120 python tools/sweep.py --ks 4 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
  for f in 0.65 0.7; do echo "rep=$rep lib=w12all split=$f ilv=2" >> $out; GOL_ILV=2 GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_w12all.so timeout -k 10 120 python tools/sweep.py --ks 12 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
done
