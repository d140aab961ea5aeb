#!/bin/bash
# The driver's bench command under rocprofv3 --kernel-trace --stats (no counters), keeping the
# per-dispatch trace (gzipped) for tools/trace_gaps.py: GPU idle time between kernels.
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-bench_trace}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 840 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?
echo "rc=$rc wall=$(( $(date +%s) - start )) s" | tee $out/wall.txt
for f in $(find $out/prof -name "*kernel_trace.csv"); do gzip -f $f; done
find $out/prof -name "*.csv*" | head
exit $rc
