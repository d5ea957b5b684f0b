#!/bin/bash
# Pair-split sweep (GOL_SPLIT) on the 65536^2 board for the default layout and depths; then the tail of
# the chosen split.   tools/split_sweep.sh out.log "fractions" "ilv:ks ..."
out=$1; fr=$2; cfgs=$3
: > $out
for rep in 1 2; do
  for f in $fr; do
    for cfg in $cfgs; do
      ilv=${cfg%%:*}; ks=${cfg#*:}
      echo "rep=$rep split=$f ilv=$ilv" >> $out
      GOL_SPLIT=$f GOL_ILV=$ilv timeout -k 10 120 python tools/sweep.py --ks $ks --passes 16 2>/dev/null | grep '^{' >> $out || exit 1
    done
  done
done
