#!/bin/bash
# prefill with sibling groups (one x quantize per group) vs one mul_mat per matrix, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/pab
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-extra --no-cpu --no-exact > gpurun_out/pab/grp.$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-extra --no-cpu --no-exact --no-batch-siblings > gpurun_out/pab/one.$r.json 2>/dev/null || exit 1
done
