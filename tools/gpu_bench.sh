#!/bin/bash
# GPU box: adamw/trainer GPU tests, then the default bench (720p x 81f PRFL iteration).
# usage: bash tools/gpu_bench.sh <tag> [bench args...]
tag=${1:-run}; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "adamw or trainer" > $out/tests.log 2>&1 || { echo tests failed; tail -20 $out/tests.log; exit 1; }
timeout -k 10 1000 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err
rc=$?
tail -3 $out/bench.err; cat $out/bench.json
exit $rc
