#!/bin/bash
# round 6: cooperative pass, two bands (workgroups) per CU (GOL_COOP_WGS=2: 8 waves per SIMD, 512 bands of 8 rows at
# 4096^2) against the shipped one per CU, at hand-off depths 4 / 6 / 8; interleaved; hashes compared
set -e
out=gpurun_out/r6v
mkdir -p $out
for rep in 1 2; do
  for w in 1 2; do
    for bd in 0 1; do
      GOL_LIB=$PWD/build/abx/libgol_coop_wgs$w.so timeout -k 10 120 python tools/coop_sweep.py --rounds 1 --boundary $bd coop_k=4,6,8 \
        | sed "s|^{|{\"wgs\": $w, |" >> $out/coop_wgs.jsonl
    done
  done
done
