#!/bin/bash
# GPU box: full GPU test suite, then the isolated 720p attention kernels.
out=gpurun_out/${1:-kern}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn_bwd 2 > $out/attnbwd720.txt 2>&1 || exit 1
PRFL_ATTN_DKDV4=1 PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn_bwd 2 > $out/attnbwd720_old.txt 2>&1 || exit 1
cat $out/attnbwd720.txt $out/attnbwd720_old.txt
