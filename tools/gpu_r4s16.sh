#!/bin/bash
# Round-4 session 16: every GEMM on the 32x32x16 four-wave kernel (GEMM_MFMA32, both kernels with
# the interleaved placement) vs the shipped split (16x16x32 for forward / dX, 32x32x16 for dW)
out=$GRAFT_REPO_ROOT/gpurun_out/r4s16; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
A=../ab
timeout -k 10 400 python ab_gemm_libs.py 256 $L $A/lib_m32il.so $L $A/lib_m32il.so --passes fwd_t,gelu_t,resid_t,dx,dgelu --reps 4 > $out/ab_gemm_m32il.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_gemm_m32il.log
