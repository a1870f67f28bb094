#!/bin/bash
# round 2: whole -m gpu suite
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r2/gpu_tests.log; exit $rc
