#!/bin/bash
# Round-4 session 10: C3 and C5 benches on the final tree
out=$GRAFT_REPO_ROOT/gpurun_out/r4s10; mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 420 python bench.py --workload prfl_t2v_480 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_prfl480.json 2> $out/bench_prfl480.err || exit $?
tail -c 400 $out/bench_prfl480.json
timeout -k 10 700 python bench.py --workload prfl_i2v_720 --fp8 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_i2v720_fp8.json 2> $out/bench_i2v720_fp8.err || exit $?
tail -c 400 $out/bench_i2v720_fp8.json
