#!/bin/bash
# Round-4 session 18: the driver's bench command on the final tree
out=$GRAFT_REPO_ROOT/gpurun_out/r4s18; mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench720.json 2> $out/bench720.err || exit $?
tail -c 1200 $out/bench720.json
