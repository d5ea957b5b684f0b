#!/bin/bash
# Interleaved A/B of library variants on the mid-size passes (tools/lanes_ab.py, one process per library and round).
#   tools/lib_ab.sh out.log reps "<lanes_ab.py args>" lib1.so lib2.so ...
out=$1; reps=$2; args=$3; shift 3
: > $out
for rep in $(seq $reps); do
  for L in "$@"; do
    GOL_LIB=$PWD/$L timeout -k 10 180 python tools/lanes_ab.py --rounds 1 $args 2>/dev/null | grep '^{' | sed "s|^{|{\"lib\": \"$(basename $L)\", \"abrep\": $rep, |" >> $out || exit 1
  done
done
