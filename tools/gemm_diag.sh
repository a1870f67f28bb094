#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gdiag
for d in ${DIAGS:-0 1 2 3 4}; do
  GGML_HIP_GEMM_DIAG=$d timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu --layers 4 > gpurun_out/gdiag/d$d.log 2>&1
  rc=$?; echo "diag=$d rc=$rc $(grep -o '"prefill": {[^}]*}' gpurun_out/gdiag/d$d.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
