#!/bin/bash
# Final verification of the tree: GPU suite, smoke(), the driver's bench command.
out=gpurun_out/${1:-s12}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash tools/gpu_bench_driver.sh ${1:-s12}/bench
