#!/bin/bash
# Forward-attention schedule A/B: SCHED 2 (current) vs 1 vs 0, three passes.
out=gpurun_out/${1:-s11}; mkdir -p $out
cd tools
for r in 1 2 3; do
timeout -k 10 300 python -u ab_attn_libs.py ../abl/alib_cur.so ../abl/alib_s1.so ../abl/alib_s0.so --reps 6 >> ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
done
grep -v amdgpu.ids ../$out/ab_attn.txt
