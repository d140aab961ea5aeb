#!/bin/bash
# Final-tree records: rocprofv3 kernel-trace + stats of the driver bench command, then the
# randomised mid_timestep bench (train_prfl.py:640-651).
tag=${1:-s15}
bash tools/gpu_rocprof_bench.sh $tag/rocprof || exit $?
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u bench.py --random-mid --no-cpu-baseline > $out/random_mid.json 2> $out/random_mid.err || { tail -20 $out/random_mid.err; exit 1; }
cat $out/random_mid.json
