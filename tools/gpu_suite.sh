#!/bin/bash
# GPU box: full GPU test suite, smoke(), then the PAVRM reward-head bench (C2, 480p).
out=gpurun_out/${1:-suite}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python -u bench.py --workload pavrm_t2v_480 --steps 3 --warmup 1 --no-cpu-baseline > $out/pavrm.json 2> $out/pavrm.err || { tail -20 $out/pavrm.err; exit 1; }
cat $out/pavrm.json
