#!/bin/bash
# Row-item GEMV with 12 / 8 waves per workgroup (variants/libggml_hip_rw*.so, -DGEMV_RW) vs 16:
# per-shape decode times (Falcon / LLaMA-13B / LLaMA-7B), 2 rounds -> gpurun_out/rw/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/rw
S="4544:4672 4544:4544 5120:5120 5120:15360 4096:4096 4096:12288 4096:22016 11008:4096 13824:5120"
run() { name=$1; shift; env "$@" timeout -k 10 120 python -u tools/shape_sweep.py $S > gpurun_out/rw/$name.log 2>&1 || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run rw12wg2_$r GGML_HIP_LIB=$PWD/variants/libggml_hip_rw12.so GGML_HIP_GEMV_WG_PER_CU=2
  run rw12_$r GGML_HIP_LIB=$PWD/variants/libggml_hip_rw12.so
  run rw8_$r GGML_HIP_LIB=$PWD/variants/libggml_hip_rw8.so
done
