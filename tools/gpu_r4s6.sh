#!/bin/bash
# Round-4 session 6: the driver's bench command on the current tree (N = 1), then C2
out=$GRAFT_REPO_ROOT/gpurun_out/r4s6; mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench720.json 2> $out/bench720.err || exit $?
tail -c 2500 $out/bench720.json
timeout -k 10 240 python bench.py --workload pavrm_t2v_480 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench_pavrm480.json 2> $out/bench_pavrm480.err || exit $?
tail -c 600 $out/bench_pavrm480.json
