#!/bin/bash
# Group-split sweep: default library at K=16 vs the 12-wave-workgroup library at K=12 (and 16-wave at K=8).
#   tools/w12_sweep.sh out.log
out=$1; : > $out
for rep in 1 2; do
  for f in 0.72 0.76 0.8; do echo "rep=$rep lib=base split=$f" >> $out; GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_base.so timeout -k 10 120 python tools/sweep.py --ks 16 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
  for f in 0.7 0.75 0.8 0.85; do echo "rep=$rep lib=w12 split=$f" >> $out; GOL_SPLIT=$f GOL_LIB=$PWD/ab/libgol_w12.so timeout -k 10 120 python tools/sweep.py --ks 8,12 --passes 16 2>/dev/null | grep '^{' >> $out || exit 1; done
done
