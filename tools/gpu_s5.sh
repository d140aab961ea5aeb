#!/bin/bash
# rocprofv3 kernel-trace + stats of the driver bench command, then PMC passes over the isolated
# 720p attention forward (split-KV tail) and the fused-epilogue GEMMs.
tag=${1:-s5}
bash tools/gpu_rocprof_bench.sh $tag/rocprof || exit $?
bash tools/pmc_kernels.sh ${tag}_attn attn 1 || exit $?
bash tools/pmc_kernels.sh ${tag}_gemmepi gemmepi 1 || exit $?
