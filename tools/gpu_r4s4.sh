#!/bin/bash
# Round-4 session 4: -m gpu suite on the VT-forward / GEMM-interleave tree, the VT read-ahead
# sweep (SCHED 2 / 3 / 5), then the PMC passes of the shipped self-attention forward
bash tools/gpu_session.sh r4s4 || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/r4s4
cd $GRAFT_REPO_ROOT/tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
A=../ab
timeout -k 10 200 python ab_attn_libs.py $A/lib_vs2.so $L $A/lib_vs5.so $A/lib_vs2.so $L $A/lib_vs5.so --qs 0,1,2,3,4,5 --vt 0,1,2,3,4,5 --reps 5 > $out/ab_fwd_vt_sched.log 2>&1 || exit $?
tail -3 $out/ab_fwd_vt_sched.log
cd $GRAFT_REPO_ROOT
timeout -k 10 400 bash tools/pmc_kernels.sh r4s4_fwd attn_l2q 1 > $out/pmc_fwd.log 2>&1 || exit $?
tail -30 $out/pmc_fwd.log
