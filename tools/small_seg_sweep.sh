#!/bin/bash
# Segment length on small boards (latency-bound): GOL_SEG_ROWS override at 1024^2 / 4096^2, ilv 1, K = 4/8.
out=$1; : > $out
for s in 1024 4096; do
  for seg in 0 4 8 12 16 32; do
    echo "size=$s seg=$seg" >> $out
    GOL_ILV=1 GOL_SEG_ROWS=$seg timeout -k 10 120 python tools/sweep.py --size $s --ks 4,8 --passes 64 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
