#!/bin/bash
# A/B on one box: streamed AdamW synchronous vs overlapped (480p workload, host moments).
out=gpurun_out/ab_opt; mkdir -p $out
for ov in 0 1 0 1; do
  PRFL_OPT_HOST=1 PRFL_OPT_OVERLAP=$ov timeout -k 10 400 python -u bench.py --workload prfl_t2v_480 --no-cpu-baseline > $out/ov$ov.json 2>> $out/err.log || exit 1
  python3 -c "import json,sys; d=json.load(open('$out/ov$ov.json')); print('overlap=$ov', d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})"
done
