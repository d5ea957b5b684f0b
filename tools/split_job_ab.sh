#!/bin/bash
# Whole-job bench (10k generations) at several group-split fractions (GOL_SPLIT), interleaved.
out=$1; : > $out
for rep in 1 2; do
  for f in 0.62 0.66 0.70 0.74; do
    echo "rep=$rep split=$f" >> $out
    GOL_SPLIT=$f timeout -k 10 200 python -u bench.py --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
