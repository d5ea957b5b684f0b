#!/bin/bash
# Depth sweep on small boards (the reference-size parity configs): latency/launch-bound regime.
out=$1; : > $out
for s in 1024 4096 16384; do
  for ilv in 1 2; do
    echo "size=$s ilv=$ilv" >> $out
    GOL_ILV=$ilv timeout -k 10 120 python tools/sweep.py --size $s --ks 1,2,4,8,12,16,32 --passes 64 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
echo "bounded 256" >> $out
timeout -k 10 120 python tools/sweep.py --size 256 --boundary 1 --ks 1,2,4,8,12,16,32 --passes 64 2>/dev/null | grep '^{' >> $out
