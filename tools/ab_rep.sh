#!/bin/bash
# Repeated, interleaved A/B of library variants on the 65536^2 board (ABAB order averages drift).
#   [AB_BOUNDARY=1] tools/ab_rep.sh out.log reps "ilv:ks ilv:ks ..." lib1.so lib2.so ...
out=$1; reps=$2; cfgs=$3; shift 3
: > $out
for rep in $(seq $reps); do
  for L in "$@"; do
    for cfg in $cfgs; do
      ilv=${cfg%%:*}; ks=${cfg#*:}
      echo "rep=$rep lib=$(basename $L) ilv=$ilv" >> $out
      GOL_LIB=$PWD/$L timeout -k 10 120 python tools/sweep.py --ilv $ilv --ks $ks --passes 16 --boundary ${AB_BOUNDARY:-0} --pre ${AB_PRE:-0} 2>/dev/null | grep '^{' >> $out || exit 1
    done
  done
done
