#!/bin/bash
# PMC comparison of prfl_gemm and hipBLASLt on the QKV forward shape (prof_kernels.py gemmcmp):
# one counter group per rocprofv3 run, each under its own time limit.
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_gemmcmp${PRFL_GEMM_TILE:+_t$PRFL_GEMM_TILE}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
export PRFL_PROF_L=73920
i=0
for p in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY" \
         "FETCH_SIZE" "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $p -d $out/p$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py gemmcmp 3 > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out | tee $out/summary.txt
