#!/bin/bash
# GPU box: A/B of the attention-output stash budget on the default 720p bench, same box.
# usage: bash tools/gpu_stash_ab.sh <tag> <gbA> <gbB>
tag=${1:-stash}; out=gpurun_out/$tag; mkdir -p $out
for gb in $2 $3; do
  PRFL_ATTN_STASH_GB=$gb timeout -k 10 700 python -u bench.py --no-cpu-baseline > $out/bench_$gb.json 2> $out/bench_$gb.err || { tail -5 $out/bench_$gb.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bench_$gb.json'));print($gb,d['ms_per_step'],d['peak_hbm_gb'],d['kernels']['attn_fwd'])"
done
