#!/bin/bash
# Round-4 probe session: backward XCD-mapping A/B, then the --pmc large-allocation probe
# (1 GB, 64 GB, 200 GB of HBM held, no training code), stopping at the first failure.
#   bash tools/gpu_r4_probe.sh <tag>
tag=${1:?tag}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log
[ $rc -ne 0 ] && exit $rc
cd $GRAFT_REPO_ROOT/tools
timeout -k 10 300 python ab_attn_libs.py ../ab/lib_abase.so ../ab/lib_axq.so ../ab/lib_axkv.so ../ab/lib_aq3.so ../ab/lib_axq3.so \
  ../ab/lib_abase.so ../ab/lib_axq.so ../ab/lib_axkv.so ../ab/lib_aq3.so ../ab/lib_axq3.so --bwd --qs 0,1,2,3,4,5,6,7,8,9 --reps 4 \
  > $out/ab_bwd_xcd.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 $out/ab_bwd_xcd.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for gb in 1 64 200; do
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $out/big$gb -o pmc --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/pmc_bigalloc_probe.py $gb > $out/big$gb.log 2>&1
  rc=$?
  echo "bigalloc $gb GB rc=$rc"; grep -v "^W2026\|^E2026" $out/big$gb.log | tail -4
  [ $rc -ne 0 ] && exit $rc
done
echo probe done
