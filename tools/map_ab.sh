#!/bin/bash
# GEMV row-mapping A/B (GGML_HIP_GEMV_MAP 0/1/2 and the default) on the shape sweep + the decode bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/map
for m in ${MAPS:--1 0 1 2}; do
  GGML_HIP_GEMV_MAP=$m timeout -k 10 300 python tools/shape_sweep.py > gpurun_out/map/s$m.log 2>&1 || exit 1
  echo "map $m: $(python3 tools/shape_parse.py gpurun_out/map/s$m.log)"
  GGML_HIP_GEMV_MAP=$m ROUNDS=1 SPECS="m$m=GGML_HIP_GEMV_DIAG=0" bash tools/gemv_ab.sh || exit 1
done
