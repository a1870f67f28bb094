#!/bin/bash
# Exact mode with the q8_0 quantize folded into the exact launch (N = 1): bitwise tests, then the
# bench's exact-mode line with the fold off / on (2 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/fold
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_parity.py -x -v --timeout 200 \
  --timeout-method thread -k "exact or golden" > gpurun_out/fold/pytest.log 2>&1 || exit 1
for r in 1 2; do
  for f in 0 1; do
    GGML_HIP_EXACT_FOLD=$f timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-prefill --no-extra \
      > gpurun_out/fold/bench_f${f}_$r.json 2> gpurun_out/fold/bench_f${f}_$r.err || exit 1
  done
done
