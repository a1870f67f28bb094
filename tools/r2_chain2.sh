#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
for d in ${DEPTHS:-2 8}; do
GGML_HIP_CHAIN_DEPTH=$d GGML_HIP_CHAIN_STAMPS=1 timeout -k 10 120 python tools/chain_stamps.py 2 > gpurun_out/r2/chain_stamps_d$d.log 2>&1
rc=$?; echo "== depth $d"; cat gpurun_out/r2/chain_stamps_d$d.log; [ $rc = 0 ] || exit $rc
done
