#!/bin/bash
# GEMV launch-shape sweep: per-shape kernel durations under rocprofv3 for several grid caps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for wg in ${WGS:-1 2}; do
  GGML_HIP_GEMV_WG_PER_CU=$wg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sweep/wg$wg -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-prefill > gpurun_out/sweep/wg$wg.log 2>&1
  rc=$?; echo "wg=$wg rc=$rc"; tail -1 gpurun_out/sweep/wg$wg.log | cut -c1-200
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
