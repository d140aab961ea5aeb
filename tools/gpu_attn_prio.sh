#!/bin/bash
# GPU box: same-box A/B of the 720p self-attention forward (pp3) over the wave-priority modes.
for i in 1 2; do
  for pr in 0 1 2; do
    PRFL_ATTN_PRIO=$pr PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 2>&1 | grep "attn_fwd:" | sed "s/^/prio$pr /" || exit 1
  done
done
