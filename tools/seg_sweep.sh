#!/bin/bash
# Segment-length sweep (GOL_SEG_ROWS) for library variants on the 65536^2 board.
#   tools/seg_sweep.sh out.log "ilv:k" "rows1 rows2 ..." lib1.so lib2.so ...
out=$1; cfg=$2; rows=$3; shift 3
ilv=${cfg%%:*}; k=${cfg#*:}
for L in "$@"; do
  for r in $rows; do
    echo "lib=$(basename $L) ilv=$ilv seg=$r" >> $out
    GOL_SEG_ROWS=$r GOL_LIB=$PWD/$L GOL_ILV=$ilv timeout -k 10 120 python tools/sweep.py --ks $k --passes 8 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
