#!/bin/bash
# GPU box: same-box A/B of the 720p self-attention forward between the current library and
# prfl_amd/lib/libprfl_hip_prev.so (the previous build), alternated; then attention parity.
for i in 1 2; do
  PRFL_HIP_LIB=$PWD/hy-video-prfl_amd/prfl_amd/lib/libprfl_hip_prev.so PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 2>&1 | grep "attn_fwd:" | sed "s/^/prev /" || exit 1
  PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 2>&1 | grep "attn_fwd:" | sed "s/^/new  /" || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_block.py -x -q --timeout 200 --timeout-method thread -k "attention or block" 2>&1 | tail -1
