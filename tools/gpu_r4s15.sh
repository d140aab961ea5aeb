#!/bin/bash
# Round-4 session 15: weight-gradient GEMM (gemm4x) with the interleaved placement vs without
out=$GRAFT_REPO_ROOT/gpurun_out/r4s15; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
A=../ab
timeout -k 10 300 python ab_gemm_libs.py 256 $A/lib_x4base.so $A/lib_x4il.so $A/lib_x4base.so $A/lib_x4il.so --passes dw,dwacc --reps 5 > $out/ab_gemm4x_il.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_gemm4x_il.log
