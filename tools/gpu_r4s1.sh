#!/bin/bash
# Round-4 session 1: -m gpu suite, then the VT/KT A/B (forward: row-major vs VT; backward:
# row-major vs KT, and the dQ ring / stagger / XCD variants built by tools/build_variant.sh)
SKIP_TESTS=${SKIP_TESTS:-0} bash tools/gpu_session.sh r4s1 || exit $?
cd tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
timeout -k 10 200 python ab_attn_libs.py $L $L $L $L --qs 0,1,2,3 --vt 1,3 --reps 6 > ../gpurun_out/r4s1/ab_fwd_vt.log 2>&1 || exit $?
tail -4 ../gpurun_out/r4s1/ab_fwd_vt.log
A=../ab
timeout -k 10 400 python ab_attn_libs.py $L $L $A/lib_abase.so $A/lib_aq3.so $A/lib_as3.so $A/lib_axq.so $L $L $A/lib_abase.so $A/lib_aq3.so $A/lib_as3.so $A/lib_axq.so --bwd --qs 0,1,2,3,4,5,6,7,8,9,10,11 --vt 1,7 --reps 3 > ../gpurun_out/r4s1/ab_bwd.log 2>&1 || exit $?
tail -4 ../gpurun_out/r4s1/ab_bwd.log
timeout -k 10 300 python ab_gemm_libs.py 256 $L $A/lib_gil.so $L $A/lib_gil.so --passes fwd,dx --reps 5 > ../gpurun_out/r4s1/ab_gemm_il.log 2>&1 || exit $?
tail -10 ../gpurun_out/r4s1/ab_gemm_il.log
