#!/bin/bash
# round 2: arch frontends (Falcon via the reference's falcon.cpp), full-size arch shapes, hook tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_falcon_arch.py tests/test_gpu_parity.py tests/test_gpu_ggml_hook.py tests/test_gpu_llama_ggjt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/arch_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r2/arch_tests.log; exit $rc
