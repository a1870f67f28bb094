#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-a b c d}; do
  for shape in "4096 4096" "4096 11008" "11008 4096"; do
    set -- $shape
    r=$(GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so GGML_HIP_GEMM_DIAG=0 K=$1 M=$2 timeout -k 10 120 python tools/gemm_stamps.py 2>&1 | grep "us per")
    rc=$?; echo "variant $v: $r"
  done
done
