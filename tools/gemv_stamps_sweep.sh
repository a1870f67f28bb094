#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
for d in 1 2 4; do for km in 4096:4096 4096:12288 11008:4096; do
  IFS=: read k m <<< "$km"
  echo "== depth $d K=$k M=$m"
  GGML_HIP_GEMV_DEPTH=$d K=$k M=$m timeout -k 10 120 python tools/gemv_stamps.py || exit $?
done; done
