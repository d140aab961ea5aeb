#!/bin/bash
# Round-4 session 13 (final tree): -m gpu suite + smoke, then the PMC passes of the shipped
# self-attention forward (the bench line's traffic source)
bash tools/gpu_session.sh r4s13 || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/r4s13
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 400 bash tools/pmc_kernels.sh r4s13_fwd attn_l2q 1 > $out/pmc_fwd.log 2>&1 || exit $?
grep -A18 "attn_fwd_kernel<false, 3, 3, true, true>" $GRAFT_REPO_ROOT/gpurun_out/pmc_r4s13_fwd/summary.txt
