#!/bin/bash
# GPU suite, then forward-attention DMA A/B and four-wave epilogue A/B (abl/*.so).
out=gpurun_out/${1:-s3}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd tools
timeout -k 10 300 python -u ab_attn_libs.py ../abl/alib0.so ../abl/alib1.so --reps 6 > ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
grep -v amdgpu.ids ../$out/ab_attn.txt
cd ..
timeout -k 10 300 python -u tools/ab_gemm_libs.py 256 abl/lib1.so abl/lib3.so abl/lib4.so abl/lib5.so --shapes ffn1 --passes gelu --reps 5 > $out/ab_gemm.txt 2>&1 || { tail -20 $out/ab_gemm.txt; exit 1; }
timeout -k 10 300 python -u tools/ab_gemm_libs.py 256 abl/lib1.so abl/lib3.so abl/lib4.so abl/lib5.so --shapes o,ffn2 --passes resid,dgelu,dwacc --reps 5 >> $out/ab_gemm.txt 2>&1 || { tail -20 $out/ab_gemm.txt; exit 1; }
grep -v amdgpu.ids $out/ab_gemm.txt
