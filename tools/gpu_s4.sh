#!/bin/bash
# GPU suite, split-KV tail A/B (abl/alib2 = no split, alib3 = split), driver bench command.
out=gpurun_out/${1:-s4}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd tools
timeout -k 10 300 python -u ab_attn_libs.py ../abl/alib2.so ../abl/alib3.so --reps 8 > ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
grep -v amdgpu.ids ../$out/ab_attn.txt
cd ..
bash tools/gpu_bench_driver.sh ${1:-s4}/bench
