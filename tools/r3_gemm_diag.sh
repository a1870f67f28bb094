#!/bin/bash
# k_gemm8 knockouts (results invalid): 81 = DMA ring + barriers only, 82 = compute only; rocprof medians
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for d in ${DIAGS:-0 81 82 83}; do
  GGML_HIP_GEMM_V=9 GGML_HIP_GEMM_DIAG=$d timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3d/d$d -o run --output-format csv -- python3 tools/gemm_shapes.py > gpurun_out/r3d/d$d.log 2>&1
  rc=$?; echo "diag $d rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  python3 tools/kt_median.py gpurun_out/r3d/d$d gemm8
done
