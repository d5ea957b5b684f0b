#!/bin/bash
# Interleaved A/B of two library builds on BASELINE config 2 (4096^2, 1000 generations per call), torus and
# bounded, `reps` rounds: tools/coop_4096_ab.sh reps lib1.so lib2.so
reps=$1; shift
for rep in $(seq $reps); do
  for L in "$@"; do
    echo "lib=$(basename $L)"
    GOL_LIB=$PWD/$L python -u tools/small_configs.py | grep -E '"w": 4096, "h": 4096' || exit 1
  done
done
