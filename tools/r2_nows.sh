#!/bin/bash
# A/B: v7 GEMM vs the same kernel with its weight staging knocked out (diagnostic, results invalid)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nows
for r in 1 2; do
  timeout -k 10 120 python -u tools/gemm_shapes.py > gpurun_out/nows/base_$r.log 2>&1
  GGML_HIP_LIB=$PWD/variants/libggml_hip_nows.so timeout -k 10 120 python -u tools/gemm_shapes.py > gpurun_out/nows/nows_$r.log 2>&1
done
