#!/bin/bash
# Chunk-balanced decode GEMV (BAL): parity tests, then per-shape timing BAL off vs auto (2 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/bal
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "balanced or arch_decode or policies or siblings or 13b or llama7b_decode" > gpurun_out/bal/pytest.log 2>&1 || exit 1
S="18176:4544 13824:5120 5120:13824 4544:18176 12352:4096 24576:6144 11008:4096"
for r in 1 2; do
  GGML_HIP_GEMV_BAL=0 timeout -k 10 120 python -u tools/shape_sweep.py $S > gpurun_out/bal/off_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/shape_sweep.py $S > gpurun_out/bal/auto_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-prefill > gpurun_out/bal/bench.json 2> gpurun_out/bal/bench.err || exit 1
