#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/diag
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for w in ${WAVES_LIST:-16}; do for d in ${DIAGS:-0 1 2 3}; do
  GGML_HIP_GEMV_WAVES=$w GGML_HIP_GEMV_DIAG=$d timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/diag/w${w}d$d -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-prefill > gpurun_out/diag/w${w}d$d.log 2>&1
  rc=$?; echo "waves=$w diag=$d rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done; done
exit 0
