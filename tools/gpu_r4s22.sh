#!/bin/bash
# Round-4 session 22: C1 (pre_480, with its CPU leg) and C2 on the final tree
out=$GRAFT_REPO_ROOT/gpurun_out/r4s22; mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --workload pre_480 --steps 20 --warmup 2 > $out/bench_c1.json 2> $out/bench_c1.err || exit $?
tail -c 500 $out/bench_c1.json
timeout -k 10 240 python bench.py --workload pavrm_t2v_480 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_pavrm480.json 2> $out/bench_pavrm480.err || exit $?
tail -c 300 $out/bench_pavrm480.json
