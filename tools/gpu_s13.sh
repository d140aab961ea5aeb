#!/bin/bash
# Four-wave GEMM persistence A/B: plib0 = one tile per workgroup, plib1 = persistent (one
# workgroup per CU), plib2 = persistent + next tile's first slices issued before the epilogue.
out=gpurun_out/${1:-s13}; mkdir -p $out
timeout -k 10 500 python -u tools/ab_gemm_libs.py 256 abl/plib0.so abl/plib1.so abl/plib2.so --shapes qkv,o,ffn1,ffn2 --passes fwd,gelu,resid,dx,dwacc --reps 4 > $out/ab_persist.txt 2>&1 || { tail -20 $out/ab_persist.txt; exit 1; }
grep -v amdgpu.ids $out/ab_persist.txt
