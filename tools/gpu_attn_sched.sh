#!/bin/bash
# GPU box: same-box A/B of the 720p self-attention forward: pp3 (96-key tiles) at SCHED 0/1/2.
for i in 1 2; do
  for sc in 1 0 2; do
    PRFL_ATTN_NKT=3 PRFL_ATTN_SCHED=$sc PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 2>&1 | grep "attn_fwd:" | sed "s/^/pp3 sched$sc /" || exit 1
  done
done
