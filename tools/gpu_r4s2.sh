#!/bin/bash
# Round-4 session 2: the driver's bench command under rocprofv3 --kernel-trace --stats (the
# per-kernel summary behind the line's roofline), then PMC passes of the shipped self-attention
# forward (the line's traffic source).  Each step under its own limit; first failure ends it.
tag=${1:-r4s2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
bash tools/gpu_bench_rocprof.sh $tag/rocprof || exit $?
tail -c 3000 $out/rocprof/bench.json
if [ "${SKIP_PMC:-0}" != "1" ]; then
  timeout -k 10 400 bash tools/pmc_kernels.sh ${tag}_fwd attn_l2q 1 > $out/pmc_fwd.log 2>&1 || exit $?
  tail -30 $out/pmc_fwd.log
fi
