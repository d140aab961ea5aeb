#!/bin/bash
# Round-4 session 11: VT forward knob re-sweep (DMA placement, lazy-rescale tau, read groups, read-ahead)
out=$GRAFT_REPO_ROOT/gpurun_out/r4s11; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
A=../ab
timeout -k 10 300 python ab_attn_libs.py $L $A/lib_g0y0.so $A/lib_tau10.so $A/lib_rg2.so $A/lib_vs4.so $L $A/lib_g0y0.so $A/lib_tau10.so $A/lib_rg2.so $A/lib_vs4.so --qs 0,1,2,3,4,5,6,7,8,9 --vt 0,1,2,3,4,5,6,7,8,9 --reps 4 > $out/ab_fwd_knobs.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_fwd_knobs.log
