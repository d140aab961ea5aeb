#!/bin/bash
# Round-1 record: a rocprofv3 --pmc pass with --kernel-include-regex over bench.py died with
# SIGSEGV at the first libprfl_hip.so launch.  Same counter, same short program, with and without
# the regex filter, each under its own limit.
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_regex; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
export PRFL_PROF_L=8192
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES -d $out/plain -o pmc --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py gemm720 1 > $out/plain.log 2>&1
echo "no regex: rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES --kernel-include-regex gemm256s -d $out/regex -o pmc \
  --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py gemm720 1 > $out/regex.log 2>&1
echo "with regex: rc=$?"
tail -3 $out/regex.log
exit 0
