#!/bin/bash
# Whole-job bench on a bounded 65536^2 board at K = 12 and 16, interleaved.
out=$1; : > $out
for rep in 1 2; do
  for k in 12 16; do
    echo "rep=$rep tblock=$k" >> $out
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --boundary bounded --tblock $k 2>/dev/null | grep '^{' >> $out || exit 1
  done
done
