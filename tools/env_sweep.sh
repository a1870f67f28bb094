#!/bin/bash
# HIP runtime dispatch switches vs the graph launch floor and the decode bench (A/B in one box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/env
for e in ${ENVS:-NONE=1 ROC_SYSTEM_SCOPE_SIGNAL=0 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_HIP_GRAPH_BATCH_SIZE=64 ROC_USE_FGS_KERNARG=0 HIP_FORCE_DEV_KERNARG=1}; do
  floor=$(env $e timeout -k 10 60 ./tools/launch_floor 2>&1 | grep "grid   512 block 1024 lds     0 touch 0 graph" | awk '{print $(NF-3)}')
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-prefill > gpurun_out/env/b.log 2>&1 || { echo "$e bench rc=$?"; tail -3 gpurun_out/env/b.log; continue; }
  echo "$e floor_us=$floor tok_s=$(tail -1 gpurun_out/env/b.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
