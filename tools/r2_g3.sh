#!/bin/bash
# round 2: whole -m gpu suite on the /opt/rocm runtime (no torch in process) + bench paths
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --force-split --steps 5 --warmup 2 --no-cpu --no-prefill --no-exact --no-extra > gpurun_out/r2/bench_torchrun1.log 2>&1
rc=$?; tail -1 gpurun_out/r2/bench_torchrun1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r2/bench_full.log 2>&1
rc=$?; tail -1 gpurun_out/r2/bench_full.log; exit $rc
