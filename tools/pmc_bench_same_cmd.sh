#!/bin/bash
# rocprofv3 --pmc passes over the bench command itself (720p, one warm-up-free iteration at
# mid_timestep 1, no CPU baseline), one counter group per run, no --kernel-include-regex:
# per-dispatch FETCH_SIZE / WRITE_SIZE of every kernel of the PRFL step in the bench process.
#   bash tools/pmc_bench_same_cmd.sh <tag>
tag=${1:?tag}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_bench_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for p in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"; do
  timeout -s KILL 600 rocprofv3 --pmc $p -d $out/p$i -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --workload prfl_t2v_720 --warmup 0 --steps 1 --mid 1 \
    --no-cpu-baseline > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc"
  if [ $rc -ne 0 ]; then grep -v "^\[bench\]" $out/p$i.log | tail -5; exit $rc; fi
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out | tee $out/summary.txt
