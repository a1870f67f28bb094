#!/bin/bash
# Round 3 prefill GEMM A/B: graph-replayed LLaMA-7B shapes (N = 512) for the GEMM versions given in
# $VERS (default "8 7"), then one rocprofv3 kernel-trace --stats pass of the first version.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in ${VERS:-8 7}; do
  echo "== GGML_HIP_GEMM_V=$v"
  GGML_HIP_GEMM_V=$v timeout -k 10 120 python3 tools/gemm_shapes.py; rc=$?
  case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
done
v=$(echo ${VERS:-8 7} | cut -d' ' -f1)
GGML_HIP_GEMM_V=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g/prof -o run --output-format csv -- python3 tools/gemm_shapes.py > gpurun_out/r3g/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/r3g/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
exit 0
