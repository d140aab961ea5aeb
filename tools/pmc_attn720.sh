#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the isolated 720p self-attention forward
# (the bench's roofline kernel): HBM-side bytes and MFMA busy.  Output: gpurun_out/pmc_<tag>.
tag=${1:-attn720}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
export PRFL_PROF_L=73920
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $p -d $out/attn_p$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py attn 1 > $out/attn_p$i.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out
