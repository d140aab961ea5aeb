#!/bin/bash
# Round-4 session 5: -m gpu suite on the transposed-forward-weight tree, then the forward GEMMs
# on W^T (MN-major B) vs W (K-major), every forward epilogue, one process
bash tools/gpu_session.sh r4s5 || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/r4s5; mkdir -p $out
cd $GRAFT_REPO_ROOT/tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
timeout -k 10 400 python ab_gemm_libs.py 256 $L $L --passes fwd,fwd_t,gelu,gelu_t,resid,resid_t,fwd,fwd_t --reps 5 > $out/ab_gemm_wt.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_gemm_wt.log
