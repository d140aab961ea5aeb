#!/bin/bash
# Bench records of the other configs on this tree: PAVRM 480p (C2), I2V 720p fp8 (C5), T2V 480p (C3).
out=gpurun_out/${1:-s8}; mkdir -p $out
timeout -k 10 400 python -u bench.py --workload pavrm_t2v_480 --steps 3 --warmup 1 --no-cpu-baseline > $out/pavrm480.json 2> $out/pavrm480.err || { tail -20 $out/pavrm480.err; exit 1; }
cat $out/pavrm480.json
timeout -k 10 600 python -u bench.py --workload prfl_i2v_720 --fp8 --no-cpu-baseline > $out/i2v720_fp8.json 2> $out/i2v720_fp8.err || { tail -20 $out/i2v720_fp8.err; exit 1; }
cat $out/i2v720_fp8.json
timeout -k 10 500 python -u bench.py --workload prfl_t2v_480 --steps 2 --no-cpu-baseline --budget-s 420 > $out/prfl480.json 2> $out/prfl480.err || { tail -20 $out/prfl480.err; exit 1; }
cat $out/prfl480.json
