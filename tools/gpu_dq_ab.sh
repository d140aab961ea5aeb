#!/bin/bash
# GPU box: parity of the 96-key dQ backward (PRFL_ATTN_DQW3=1), then a same-box A/B at 720p.
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_block.py -x -q --timeout 200 --timeout-method thread -k "attention or block" 2>&1 | tail -1
for i in 1 2; do
  PRFL_ATTN_DQ64=1 PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn_bwd 2 2>&1 | grep "attn_bwd_dq:" | sed "s/^/dq8  /" || exit 1
  PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn_bwd 2 2>&1 | grep "attn_bwd_dq:" | sed "s/^/dq8w3/" || exit 1
done
