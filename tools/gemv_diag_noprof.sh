#!/bin/bash
# bench decode tok/s (no profiler) for GEMV diagnostic variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/diagnp
export PYTHONUNBUFFERED=1
for w in ${WAVES_LIST:-16}; do for d in ${DIAGS:-0 3}; do
  GGML_HIP_GEMV_WAVES=$w GGML_HIP_GEMV_DIAG=$d timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu --no-prefill > gpurun_out/diagnp/w${w}d$d.log 2>&1
  rc=$?; echo "waves=$w diag=$d rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/diagnp/w${w}d$d.log) $(grep -o '"4096->4096": {[^}]*}' gpurun_out/diagnp/w${w}d$d.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done
exit 0
