#!/bin/bash
# Round-4 session 9: -m gpu suite on the bf16-LRM tree, then the driver's bench command
bash tools/gpu_session.sh r4s9 || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/r4s9
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench720.json 2> $out/bench720.err || exit $?
tail -c 1500 $out/bench720.json
