#!/bin/bash
# Round-4 session 3: VT forward re-A/B after the read-schedule fix (+ the transpose alone), GEMM
# placement variants (IL 0 / 1 / 2)
out=$GRAFT_REPO_ROOT/gpurun_out/r4s3; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
A=../ab
timeout -k 10 200 python ab_attn_libs.py $L $L $L $L --qs 0,1,2,3 --vt 1,3 --reps 6 > $out/ab_fwd_vt.log 2>&1 || exit $?
tail -4 $out/ab_fwd_vt.log
timeout -k 10 300 python ab_gemm_libs.py 256 $A/lib_gil0.so $L $A/lib_gil2.so $A/lib_gil0.so $L $A/lib_gil2.so --passes fwd,dx --reps 5 > $out/ab_gemm_il.log 2>&1 || exit $?
tail -10 $out/ab_gemm_il.log
