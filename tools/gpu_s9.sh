#!/bin/bash
# GEMM tile-grouping A/B (GEMM_GROUP_M = 2 / 4 / 8 / 16 row blocks per XCD group), 720p shapes.
out=gpurun_out/${1:-s9}; mkdir -p $out
timeout -k 10 500 python -u tools/ab_gemm_libs.py 256 abl/glib_gm2.so abl/glib_gm4.so abl/glib_gm8.so abl/glib_gm16.so --shapes qkv,o,ffn1,ffn2 --passes fwd,resid,dx,dwacc --reps 4 > $out/ab_gm.txt 2>&1 || { tail -20 $out/ab_gm.txt; exit 1; }
grep -v amdgpu.ids $out/ab_gm.txt
