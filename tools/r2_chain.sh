#!/bin/bash
# round 2: decode-chain tests, then chain vs per-launch graph at LLaMA-7B shapes per ring depth
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2/chain_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r2/chain_tests.log; [ $rc = 0 ] || exit $rc
for d in ${DEPTHS:-8 4 2 6}; do
  GGML_HIP_CHAIN_DEPTH=$d timeout -k 10 120 python tools/chain_bench.py 32 20 > gpurun_out/r2/chain_bench_d$d.log 2>&1
  rc=$?; tail -1 gpurun_out/r2/chain_bench_d$d.log; [ $rc = 0 ] || exit $rc
done
