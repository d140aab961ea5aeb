#!/bin/bash
# GPU box: rocprofv3 kernel-trace + stats of the default bench command (no CPU baseline).
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-rocprof}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?
cat $out/bench.json; ls -R $out/prof | head -20
exit $rc
