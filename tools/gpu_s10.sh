#!/bin/bash
# Forward-attention variant A/B: current, two partial row sums, SCHED 1, SCHED 3 (two passes).
out=gpurun_out/${1:-s10}; mkdir -p $out
cd tools
for r in 1 2; do
timeout -k 10 300 python -u ab_attn_libs.py ../abl/alib_cur.so ../abl/alib_v1.so ../abl/alib_s1.so ../abl/alib_s3.so --reps 6 >> ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
done
grep -v amdgpu.ids ../$out/ab_attn.txt
