#!/bin/bash
# Round-4 measurement session (one gpurun call): PMC passes over the shipped attention kernels,
# the bench-process PMC discrimination (tools/pmc_bench_discriminate.sh), then the C2 / C3
# benches.  Each step under its own limit; the first non-zero exit ends the session.
#   bash tools/gpu_r4_measure.sh <tag>
tag=${1:?tag}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 $lim "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 $out/$name.log | cut -c1-400
  return $rc
}
if [ "${SKIP_PMC:-0}" != "1" ]; then
  step pmc_fwd 200 bash tools/pmc_kernels.sh ${tag}_fwd attn_l2q 1 || exit $?
  step pmc_bwd 240 bash tools/pmc_kernels.sh ${tag}_bwd attn_bwd_l2q 1 || exit $?
fi
if [ "${SKIP_DISC:-0}" != "1" ]; then
  step pmc_disc 700 bash tools/pmc_bench_discriminate.sh $tag || exit $?
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  step bench_pavrm480 300 python bench.py --workload pavrm_t2v_480 --steps 5 --warmup 1 || exit $?
  step bench_prfl480 420 python bench.py --workload prfl_t2v_480 --steps 2 --warmup 1 || exit $?
fi
echo session done
