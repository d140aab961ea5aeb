#!/bin/bash
# GPU box: isolated self-attention forward rate vs sequence length (480p 32760, aligned 32768, 720p 73920).
out=gpurun_out/${1:-attnL}; mkdir -p $out
for L in 32760 32768 49152 73920; do
  PRFL_PROF_L=$L timeout -k 10 120 python3 tools/prof_kernels.py attn 3 > $out/attn_$L.txt 2>&1 || { cat $out/attn_$L.txt; exit 1; }
  echo "L=$L"; cat $out/attn_$L.txt
done
