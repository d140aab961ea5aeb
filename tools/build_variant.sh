#!/bin/bash
# Build an A/B variant of libprfl_hip.so with extra -D flags into ab/lib_<name>.so (objects in
# ab/<name>/, listed in .gpurunignore; the .so travels to the GPU box):
#   bash tools/build_variant.sh <name> -DFLAG=1 ...
name=${1:?name}; shift
root=$(cd $(dirname $0)/.. && pwd)
mkdir -p $root/ab/$name
cd $root/hy-video-prfl_amd
rm -f $root/ab/$name/*.o $root/ab/lib_$name.so
pids=()
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Icsrc "$@" \
    -c $f -o $root/ab/$name/$(basename $f .hip).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "build of ab/lib_$name.so FAILED"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $root/ab/lib_$name.so $root/ab/$name/*.o
true   # object dirs stay home: .gpurunignore lists *.o
echo "built ab/lib_$name.so"
