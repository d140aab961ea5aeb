#!/bin/bash
# GPU box: full GPU test suite, then the I2V 720p x 81f PRFL bench (C5 config, bf16).
out=gpurun_out/${1:-i2v}; mkdir -p $out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 1000 python -u bench.py --workload prfl_i2v_720 --no-cpu-baseline $BENCH_EXTRA > $out/bench.json 2> $out/bench.err
rc=$?
tail -5 $out/bench.err; cat $out/bench.json
exit $rc
