#!/bin/bash
# split-K GEMM: ring depth (DP) x waves per workgroup (SK) sweep over N (tools/n_sweep.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sk
for cfg in ${CFGS:-"2 0" "4 8" "2 8" "2 16"}; do set -- $cfg
  GGML_HIP_GEMM_SK_DP=$1 GGML_HIP_GEMM_SK=$2 timeout -k 10 200 python tools/n_sweep.py ${KM:-4096 4096} > gpurun_out/sk/$1_$2.log 2>&1 || exit 1
  echo "dp $1 sk $2: $(python3 tools/sk_parse.py gpurun_out/sk/$1_$2.log)"
done
