#!/bin/bash
# Builds variants/libggml_hip_NAME.so with extra -D flags on one kernel file (A/B experiments):
#   [FILE=q4_0_gemv] bash tools/build_variant.sh xwf0 -DGEMV_XWF=0
# (the other objects come from the in-tree build: run `make -C llama.cpp-q_4_0_amd` first)
set -e
cd "$(dirname "$0")/../llama.cpp-q_4_0_amd"
name=$1; shift
file=${FILE:-q4_0_gemv}
mkdir -p ../variants/obj_$name
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -I../include"
$H ${NOKFLAGS:-$(sed -n "s/^KFLAGS *= *//p" Makefile)} "$@" -c csrc/$file.hip -o ../variants/obj_$name/$file.o
objs=""
for o in build/*.o; do
  [ "$(basename $o .o)" = "$file" ] && objs="$objs ../variants/obj_$name/$file.o" || objs="$objs $o"
done
# same identity as the in-tree library (Makefile LDIDENT): SONAME libggml_hip.so, only ggml_* exported,
# so a variant loaded by GGML_HIP_LIB is the one copy the shim's NEEDED libggml_hip.so resolves to
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/libggml_hip_$name.so $objs \
    -L/opt/rocm/lib -lrccl -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libggml_hip.so -Wl,--version-script,$PWD/exports.map
rm -rf ../variants/obj_$name
