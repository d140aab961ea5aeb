#!/bin/bash
# Round-4 session 12: 512-key cross-attention on 64-key tiles (ATTN_SHORT_NKT2) vs 96-key tiles
out=$GRAFT_REPO_ROOT/gpurun_out/r4s12; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
A=../ab
timeout -k 10 300 python ab_attn_libs.py $L $A/lib_sn2.so $L $A/lib_sn2.so --lk 512 --qs 0,1,2,3 --reps 20 > $out/ab_short.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_short.log
