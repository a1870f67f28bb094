#!/bin/bash
# Exact-mode ring depth (-DEX_SLOTS=2/4 variants vs 3): bitwise tests on each, then the bench's exact line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out/exs
for v in s2 s4; do
  GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/exs/pytest_$v.log 2>&1 || exit 1
done
for r in 1 2; do
  for v in base s2 s4; do
    lib=""; [ $v = base ] || lib="GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so"
    env $lib timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-prefill --no-extra --no-cpu \
      > gpurun_out/exs/$v.$r.json 2> gpurun_out/exs/$v.$r.err || exit 1
  done
done
