#!/bin/bash
# Interleaved A/B of library builds over the single board (torus, tools/sweep.py) and the ghost-row strip +
# bounded variants (tools/strip_sweep.py), M = 2.
#   tools/ab_all.sh out.log reps ks lib1.so lib2.so ...
out=$1; reps=$2; ks=$3; shift 3
: > $out
for rep in $(seq $reps); do
  for L in "$@"; do
    echo "rep=$rep lib=$(basename $L)" >> $out
    GOL_LIB=$PWD/$L timeout -k 10 120 python tools/sweep.py --ks $ks --passes 16 2>/dev/null | grep '^{' >> $out || exit 1
    GOL_LIB=$PWD/$L timeout -k 10 120 python tools/strip_sweep.py --ks $ks --passes 16 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
