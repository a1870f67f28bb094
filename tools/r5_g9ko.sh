#!/bin/bash
# k_gemm9 knockouts (variants/libggml_hip_g9ko*.so): per-call time of one prefill mul_mat (x image + GEMM)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in ${LIBS:-base g9ko1 g9ko3 g9ko4}; do
    for km in "4096 4096" "4096 11008" "11008 4096"; do
      set -- $km
      out=$(K=$1 M=$2 GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 60 python tools/gemm_one.py 2>&1) || { echo "$v $km rc=$?: $out"; exit 1; }
      echo "$v $out"
    done
  done
done
