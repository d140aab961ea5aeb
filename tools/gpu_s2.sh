#!/bin/bash
# GPU suite + smoke, GELU/RESID/dGELU epilogue A/B (abl/lib*.so), then the driver's bench command.
out=gpurun_out/${1:-s2}; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u tools/ab_gemm_libs.py 256 abl/lib0.so abl/lib1.so abl/lib2.so --shapes ffn1 --passes gelu --reps 5 > $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }
timeout -k 10 300 python -u tools/ab_gemm_libs.py 256 abl/lib0.so abl/lib1.so abl/lib2.so --shapes o,ffn2 --passes resid,dgelu --reps 5 >> $out/ab.txt 2>&1 || { tail -20 $out/ab.txt; exit 1; }
grep -v amdgpu.ids $out/ab.txt
bash tools/gpu_bench_driver.sh ${1:-s2}/bench
