#!/bin/bash
# GPU box: parity of the 96-key-tile attention forward (PRFL_ATTN_NKT=3), then a same-box A/B of
# the isolated 720p self-attention forward, pp2 (64-key tiles) vs pp3 (96-key tiles), alternated.
out=gpurun_out/${1:-nkt}; mkdir -p $out
PRFL_ATTN_NKT=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_block.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "attention or block or wanmodel or flash" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 2>&1 | grep "attn_fwd:" | sed "s/^/pp2 /" || exit 1
  PRFL_ATTN_NKT=3 PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 2>&1 | grep "attn_fwd:" | sed "s/^/pp3 /" || exit 1
done
