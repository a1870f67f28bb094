#!/bin/bash
# k_gemm8 VAR sweep (GGML_HIP_GEMM8_VAR), 2 interleaved rounds, kernel medians from rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3v
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in ${VARS:-0 1 2 3}; do
    GGML_HIP_GEMM_V=9 GGML_HIP_GEMM8_VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3v/v$v.$r -o run --output-format csv -- python3 tools/gemm_shapes.py > gpurun_out/r3v/v$v.$r.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
    echo "VAR $v round $r"; python3 tools/kt_median.py gpurun_out/r3v/v$v.$r gemm8
  done
done
