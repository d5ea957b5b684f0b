#!/bin/bash
# Whole-job bench (10k generations) at several temporal depths, interleaved.
out=$1; : > $out
for rep in 1 2; do
  for k in 12 16; do
    echo "rep=$rep tblock=$k" >> $out
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --tblock $k 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
