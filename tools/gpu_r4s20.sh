#!/bin/bash
# Round-4 session 20: static priority for waves 4-7 in the backward kernels (ATTN_BWD_PRIO 0-3)
out=$GRAFT_REPO_ROOT/gpurun_out/r4s20; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
A=../ab
timeout -k 10 400 python ab_attn_libs.py $A/lib_bp0.so $A/lib_bp1.so $A/lib_bp2.so $A/lib_bp3.so $A/lib_bp0.so $A/lib_bp1.so $A/lib_bp2.so $A/lib_bp3.so --bwd --qs 0,1,2,3,4,5,6,7 --reps 3 > $out/ab_bwd_prio.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_bwd_prio.log
