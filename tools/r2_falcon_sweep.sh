#!/bin/bash
# Falcon-7B decode shapes (BASELINE config 5) under the GEMV policy knobs: which launch is slow, and
# does another policy fix it?  -> gpurun_out/fsweep/*.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/fsweep
S="4544:4672 4544:4544 4544:18176 18176:4544 4096:4096 4096:11008"
run() { name=$1; shift; env "$@" timeout -k 10 120 python -u tools/shape_sweep.py $S > gpurun_out/fsweep/$name.log 2>&1 || exit 1; }
run base
run var3 GGML_HIP_GEMV_VAR=3
run var15 GGML_HIP_GEMV_VAR=15
run map0 GGML_HIP_GEMV_MAP=0
run map1 GGML_HIP_GEMV_MAP=1
run map2 GGML_HIP_GEMV_MAP=2
run wg1 GGML_HIP_GEMV_WG_PER_CU=1
run wg2 GGML_HIP_GEMV_WG_PER_CU=2
run d1 GGML_HIP_GEMV_DEPTH=1
run d2 GGML_HIP_GEMV_DEPTH=2
run norow GGML_HIP_GEMV_ROWITEMS=0
run base2
