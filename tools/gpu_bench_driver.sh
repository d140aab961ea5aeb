#!/bin/bash
# The driver's exact bench command, under its 600 s limit; JSON line + stderr under gpurun_out/.
out=gpurun_out/${1:-bench}
mkdir -p $out
start=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${@:2} > $out/bench.json 2> $out/bench.err
rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start )) s" | tee $out/wall.txt
tail -5 $out/bench.err
cat $out/bench.json
exit $rc
