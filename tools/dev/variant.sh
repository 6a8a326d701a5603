#!/bin/bash
# Dev (CPU): build an A/B variant of libgcslam.so with extra -D flags on one source file.
# Usage: bash tools/dev/variant.sh <name> <source (.hip or .cpp, no suffix)> <flags...>  ->  fl-slam_amd/build_var/<name>/libgcslam.so
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../../fl-slam_amd"
d=build_var/$name; mkdir -p $d
f=csrc/$src.hip; [ -f $f ] || f=csrc/$src.cpp
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" -c $f -o $d/$src.o
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $d/$src.o -o $d/libgcslam.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $d/libgcslam.so
