#!/bin/bash
# round 2 (re-entry): whole -m gpu suite, smoke, default bench, rocprofv3 kernel stats of the eager bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r2/smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2/bench_full.log 2>&1
rc=$?; tail -1 gpurun_out/r2/bench_full.log; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2/prof_eager -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --eager --steps 20 --warmup 5 --no-cpu --no-extra > $GRAFT_REPO_ROOT/gpurun_out/r2/bench_prof_eager.log 2>&1
rc=$?; tail -1 $GRAFT_REPO_ROOT/gpurun_out/r2/bench_prof_eager.log; exit $rc
