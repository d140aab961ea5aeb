#!/bin/bash
# Round-4 session 21: GEMM tile grouping (GEMM_GROUP_M 2 / 4 / 8) on the W^T forward GEMMs
out=$GRAFT_REPO_ROOT/gpurun_out/r4s21; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
A=../ab
timeout -k 10 400 python ab_gemm_libs.py 256 $A/lib_gg4.so $A/lib_gg2.so $A/lib_gg8.so $A/lib_gg4.so $A/lib_gg2.so $A/lib_gg8.so --passes fwd_t,resid_t,dx --reps 4 > $out/ab_gemm_group.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_gemm_group.log
