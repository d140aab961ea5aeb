#!/bin/bash
# GPU box: attention GPU tests, then isolated 720p attention forward A/B (env-selected kernels).
out=gpurun_out/${1:-attn_ab}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or block" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in ${VARIANTS:-"PRFL_ATTN_PP1=1" "X=1"}; do
  env $v PRFL_PROF_L=73920 timeout -k 10 120 python3 tools/prof_kernels.py attn 3 > $out/a.txt 2>&1 || exit 1
  echo "$v $(grep attn_fwd: $out/a.txt)"
done
