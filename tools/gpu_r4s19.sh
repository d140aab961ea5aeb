#!/bin/bash
# Round-4 session 19: dK/dV scheduling fences (ATTN_DKDV_SB 0 / 1 / 2 / 3)
out=$GRAFT_REPO_ROOT/gpurun_out/r4s19; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
A=../ab
timeout -k 10 400 python ab_attn_libs.py $A/lib_dsb3.so $A/lib_dsb0.so $A/lib_dsb1.so $A/lib_dsb2.so $A/lib_dsb3.so $A/lib_dsb0.so $A/lib_dsb1.so $A/lib_dsb2.so --bwd --qs 0,1,2,3,4,5,6,7 --reps 3 > $out/ab_dkdv_sb.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_dkdv_sb.log
