#!/bin/bash
# Build lib/libpqgpu_<name>.so: kernels.hip (and bytearray.hip) compiled with extra -D flags,
# linked with the other objects of the default build (A/B runs of kernel variants in one session; experiments only).
set -e
name=$1; shift
cd "$(dirname "$0")/../parquet-go-1_amd"
make -s all
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F "$@" -c csrc/kernels.hip -o build/kernels_$name.o &
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F "$@" -c csrc/bytearray.hip -o build/bytearray_$name.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libpqgpu_$name.so build/kernels_$name.o build/bytearray_$name.o \
  build/nested.o build/pagewalk.o build/plainba.o build/host.o build/format.o build/pipeline.o -lz -lpthread
echo lib/libpqgpu_$name.so
