#!/bin/bash
# k_gemm9 knockouts (GGML_HIP_GEMM_DIAG 91 no compute / 92 no DMA / 93 no DMA, no barrier), kernel medians
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3g9d
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for d in ${DIAGS:-0 91 92 93}; do
  GGML_HIP_GEMM_V=11 GGML_HIP_GEMM_DIAG=$d timeout -k 10 200 rocprofv3 --kernel-trace -d $O/d$d -o run --output-format csv -- python3 tools/gemm_shapes.py > $O/d$d.log 2>&1
  rc=$?; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
  echo "DIAG $d"; python3 tools/kt_median.py $O/d$d k_gemm9
done
