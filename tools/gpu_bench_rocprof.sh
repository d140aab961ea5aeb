#!/bin/bash
# The driver's bench command under rocprofv3 --kernel-trace --stats (no counters): the per-kernel
# summary behind bench.py's roofline (average launch duration of the dominant kernel).
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-bench_rocprof}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 840 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start )) s" | tee $out/wall.txt
find $out/prof -name "*kernel_stats.csv" | head -3
exit $rc
