#!/bin/bash
# rocprofv3 --pmc passes over the BENCH PROCESS itself on config C1 (bench.py --workload pre_480:
# the fused 14B block forward, no grad: every dispatch from the main thread, which is what counter
# collection survives -- profiles/r05_pmc_notes.txt).  One counter group per run:
#   bash tools/pmc_bench_c1.sh <tag>  -> gpurun_out/pmc_<tag>/summary.txt (CSV files removed)
tag=${1:?tag}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  timeout -s KILL 240 rocprofv3 --pmc $p -d $out/p$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --workload pre_480 --steps 3 --warmup 1 --no-cpu-baseline > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ne 0 ]; then grep -v "^W2026\|^I2026\|^E2026" $out/p$i.log | tail -5; exit $rc; fi
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out > $out/summary.txt && rm -rf $out/p0 $out/p1 $out/p2
cat $out/summary.txt
