#!/bin/bash
# GPU box: one rocprofv3 --pmc pass over the default bench (one iteration, no warmup), counters of
# the self-attention forward only -> effective clock (GRBM_GUI_ACTIVE) and MFMA busy in the bench,
# to compare with the isolated kernel (profiles/r01_pmc_attn_fwd720_v4.txt).
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcbench}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 900 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex attn_fwd_kernel -d $out/prof -o bench --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --warmup 0 --steps 1 > $out/bench.json 2> $out/bench.err
rc=$?
cat $out/bench.json; ls -R $out/prof | head
exit $rc
