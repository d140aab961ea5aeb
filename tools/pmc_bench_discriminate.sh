#!/bin/bash
# Which part of the bench process makes `rocprofv3 --pmc` fault (profiles/r03_pmc_bench_notes.txt:
# SIGSEGV in the profiler's dispatch interception at the first clip_grad_norm_ launch of the 720p
# bench, round 3)?  One counter (FETCH_SIZE) per run, each under its own time limit; stops at the
# first failure.
#   1. --toy: the 720p memory plan's code paths (optimizer side stream, pinned-host AdamW moments
#      on a copy stream, cross-stream events, attention stash) on a 2-block 256-wide model: every
#      stream of the 720p process, a few hundred MB of HBM;
#   2. --workload prfl_t2v_480: the 14B model at 480p x 81f, moments in HBM (no copy stream, no
#      pinned host memory), ~250 GB of HBM allocated;
#   3. (only with FULL=1) the 720p command itself.
#   bash tools/pmc_bench_discriminate.sh <tag>
tag=${1:?tag}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_disc_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {   # name, time limit, bench args...
  local name=$1 lim=$2; shift 2
  timeout -s KILL $lim rocprofv3 --pmc FETCH_SIZE -d $out/$name -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep -v "^\[bench\]" $out/$name.log | tail -3
  return $rc
}
run toy 240 --toy --warmup 1 --steps 2 --no-cpu-baseline || exit $?
run prfl480 420 --workload prfl_t2v_480 --warmup 0 --steps 1 --mid 1 --no-cpu-baseline || exit $?
if [ "${FULL:-0}" = "1" ]; then
  run prfl720 600 --workload prfl_t2v_720 --warmup 0 --steps 1 --mid 1 --no-cpu-baseline || exit $?
fi
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out > $out/summary.txt
echo done
