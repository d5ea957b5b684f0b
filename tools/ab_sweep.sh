#!/bin/bash
# A/B sweep of library variants x layouts on the 65536^2 board (one process per variant/layout).
#   tools/ab_sweep.sh out.log lib1.so lib2.so ...
out=$1; shift
: > $out
for L in "$@"; do
  for cfg in "1:16,24" "2:8,12,16" "4:4,6,8"; do
    ilv=${cfg%%:*}; ks=${cfg#*:}
    echo "lib=$(basename $L) ilv=$ilv" >> $out
    GOL_LIB=$PWD/$L GOL_ILV=$ilv timeout -k 10 120 python tools/sweep.py --ks $ks --passes 8 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
