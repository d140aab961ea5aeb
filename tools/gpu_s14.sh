#!/bin/bash
# GPU suite (split tails fwd + bwd), backward split-tail A/B (alib_cur = forward split only,
# alib_bsplit = + dK/dV and dQ split tails), the driver bench command.
out=gpurun_out/${1:-s14}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd tools
timeout -k 10 400 python -u ab_attn_libs.py ../abl/alib_cur.so ../abl/alib_bsplit.so --reps 4 --bwd > ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
grep -v amdgpu.ids ../$out/ab_attn.txt
cd ..
bash tools/gpu_bench_driver.sh ${1:-s14}/bench
