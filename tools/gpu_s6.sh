#!/bin/bash
# GPU suite; attention A/Bs (alib2 = no split vs alib3 = split-KV tail, forward;
# alib3 vs alib5 = dQ DMA offsets re-derived per tile, backward); the driver bench command.
out=gpurun_out/${1:-s6}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cd tools
timeout -k 10 300 python -u ab_attn_libs.py ../abl/alib2.so ../abl/alib3.so --reps 8 > ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
timeout -k 10 400 python -u ab_attn_libs.py ../abl/alib3.so ../abl/alib5.so --reps 4 --bwd >> ../$out/ab_attn.txt 2>&1 || { tail -20 ../$out/ab_attn.txt; exit 1; }
grep -v amdgpu.ids ../$out/ab_attn.txt
cd ..
bash tools/gpu_bench_driver.sh ${1:-s6}/bench
