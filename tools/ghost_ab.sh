#!/bin/bash
# Interleaved A/B of the ghost-row strip variant (multi-GPU rank interior) between library builds.
#   tools/ghost_ab.sh out.log reps ks lib1.so lib2.so ...
out=$1; reps=$2; ks=$3; shift 3
: > $out
for rep in $(seq $reps); do
  for L in "$@"; do
    echo "rep=$rep lib=$(basename $L)" >> $out
    GOL_LIB=$PWD/$L timeout -k 10 120 python tools/strip_sweep.py --ks $ks --passes 16 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
