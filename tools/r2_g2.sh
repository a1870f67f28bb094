#!/bin/bash
# round 2: split tests (loopback R=2..8, 13B shard shapes), full -m gpu suite, bench split paths
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_ggml_hook.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2/split_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2/split_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --force-split --steps 5 --warmup 2 --no-cpu --no-prefill --no-exact --no-extra > gpurun_out/r2/bench_forcesplit.log 2>&1
rc=$?; tail -2 gpurun_out/r2/bench_forcesplit.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --force-split --steps 5 --warmup 2 --no-cpu --no-prefill --no-exact --no-extra > gpurun_out/r2/bench_torchrun1.log 2>&1
rc=$?; tail -2 gpurun_out/r2/bench_torchrun1.log; exit $rc
