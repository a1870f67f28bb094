#!/bin/bash
# k_gemm9 VAR sweep (GGML_HIP_GEMM9_VAR) beside k_gemm8 (version 9), 2 interleaved rounds, kernel medians
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3g9v
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in ${VARS:-g8 0 1 2 3}; do
    if [ "$v" = g8 ]; then ver=9; else ver=11; fi
    GGML_HIP_GEMM_V=$ver GGML_HIP_GEMM9_VAR=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $O/v$v.$r -o run --output-format csv -- python3 tools/gemm_shapes.py > $O/v$v.$r.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
    echo "VAR $v round $r"; python3 tools/kt_median.py $O/v$v.$r "k_gemm"
  done
done
