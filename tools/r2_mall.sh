#!/bin/bash
# round 2: decode rate when the weight stack fits the Infinity Cache (layers 1/2) vs HBM (32), then
# rocprofv3 kernel stats of the eager bench (graph launches crash rocprofv3 on the /opt/rocm 7.2 runtime)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
for L in 1 2 4 32; do
  timeout -k 10 120 python bench.py --layers $L --steps 200 --warmup 20 --no-cpu --no-prefill --no-exact --no-extra > gpurun_out/r2/mall_L$L.log 2>&1 || exit $?
  echo "L=$L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2/mall_L$L.log) $(grep -o '"per_shape": {[^}]*}[^}]*}[^}]*}[^}]*}' gpurun_out/r2/mall_L$L.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2/prof_eager -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --eager --steps 20 --warmup 5 --no-cpu --no-extra > $GRAFT_REPO_ROOT/gpurun_out/r2/bench_prof_eager.log 2>&1
rc=$?; tail -1 $GRAFT_REPO_ROOT/gpurun_out/r2/bench_prof_eager.log; exit $rc
