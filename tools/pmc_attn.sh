#!/bin/bash
# PMC counter passes over the isolated 480p attention kernels (tools/prof_kernels.py).
# usage (on the GPU box, from the repo root): bash tools/pmc_attn.sh <tag> [which...]
tag=${1:-r01}; shift
which=${@:-attn attn_bwd}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $out/counters.txt 2>&1 || true
passes=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
        "FETCH_SIZE"
        "WRITE_SIZE"
        "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE")
[ -n "$PMC_PASSES" ] && passes=("${passes[@]:$PMC_PASSES}")
for w in $which; do
  i=0
  for p in "${passes[@]}"; do
    timeout -k 10 120 rocprofv3 --pmc $p -d $out/${w}_p$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py $w 1 > $out/${w}_p$i.log 2>&1
    rc=$?
    echo "$w pass $i rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
    i=$((i+1))
  done
done
