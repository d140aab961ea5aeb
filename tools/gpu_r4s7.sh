#!/bin/bash
# Round-4 session 7: -m gpu suite + smoke on the current tree, then the epilogue read-ahead A/B
# (EPI4_AHEAD 2 / 3) of the W^T forward GEMMs
bash tools/gpu_session.sh r4s7 || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/r4s7
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
cd tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
A=../ab
timeout -k 10 300 python ab_gemm_libs.py 256 $L $A/lib_ea2.so $L $A/lib_ea2.so --passes resid_t,gelu_t,fwd_t --reps 5 > $out/ab_gemm_ahead.log 2>&1 || exit $?
grep -v amdgpu.ids $out/ab_gemm_ahead.log
