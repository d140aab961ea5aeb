#!/bin/bash
# rocprofv3 --pmc passes (one counter group per run, each under its own time limit, no
# --kernel-include-regex: see profiles/r02_pmc_notes.txt) over isolated 720p hot kernels:
#   bash tools/pmc_kernels.sh <tag> <prof_kernels.py workload> [reps]
# -> gpurun_out/pmc_<tag>/p*/ + summary.txt (per-kernel mean per dispatch).
tag=${1:?tag}; wl=${2:?workload}; reps=${3:-1}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
export PRFL_PROF_L=${PRFL_PROF_L:-73920}
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  timeout -s KILL 150 rocprofv3 --pmc $p -d $out/p$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py $wl $reps > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out | tee $out/summary.txt
