#!/bin/bash
# GEMV launch-policy knobs over the bench's four LLaMA-7B launch shapes (fused siblings as one matrix of
# the summed rows: same grid and row mapping as the multi launch) -> gpurun_out/lsweep/*.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/lsweep
S="4096:12288 4096:4096 4096:22016 11008:4096"
run() { name=$1; shift; env "$@" timeout -k 10 120 python -u tools/shape_sweep.py $S > gpurun_out/lsweep/$name.log 2>&1 || exit 1; }
for r in 1 2; do
  run base_$r X=1
  run map0_$r GGML_HIP_GEMV_MAP=0
  run map1_$r GGML_HIP_GEMV_MAP=1
  run map2_$r GGML_HIP_GEMV_MAP=2
  run wg1_$r GGML_HIP_GEMV_WG_PER_CU=1
  run wg2_$r GGML_HIP_GEMV_WG_PER_CU=2
  run wg1m0_$r GGML_HIP_GEMV_WG_PER_CU=1 GGML_HIP_GEMV_MAP=0
done
