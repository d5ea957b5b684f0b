#!/bin/bash
# Whole-job bench (10k generations) for library variants, interleaved: tools/variant_job_ab.sh out lib...
out=$1; shift; : > $out
for rep in 1 2; do
  for L in "$@"; do
    echo "rep=$rep lib=$L" >> $out
    GOL_LIB=$PWD/ab/libgol_$L.so timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
