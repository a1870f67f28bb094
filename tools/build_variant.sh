#!/bin/bash
# Builds variants/libggml_hip_NAME.so with extra -D flags on the kernel file (A/B experiments):
#   bash tools/build_variant.sh ws4 -DGEMV_WSLEEP=4
set -e
cd "$(dirname "$0")/../llama.cpp-q_4_0_amd"
name=$1; shift
mkdir -p ../variants/obj_$name
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -I../include"
$H ${NOKFLAGS:-$(sed -n "s/^KFLAGS *= *//p" Makefile)} "$@" -c csrc/q4_0_kernels.hip -o ../variants/obj_$name/q4_0_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/libggml_hip_$name.so build/ggml-hip.o build/ggml-hip-graph.o \
    ../variants/obj_$name/q4_0_kernels.o build/q4_0_chain.o build/ggml_ops.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf ../variants/obj_$name
