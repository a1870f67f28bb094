#!/bin/bash
# Interleaved A/B of whole-library variants (variants/libggml_hip_NAME.so, tools/build_variant.sh):
# per round and variant, the prefill GEMM shapes (tools/gemm_shapes.py) and the decode bench line.
#   LIBS="base noslp" ROUNDS=2 bash tools/lib_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    lib=$PWD/variants/libggml_hip_$v.so
    if [ -z "$NO_GEMM" ]; then
      GGML_HIP_LIB=$lib timeout -k 10 120 python tools/gemm_shapes.py > gpurun_out/ab/gemm_$v.$r.log 2>&1 || { echo "gemm $v rc=$?"; exit 1; }
      echo "$v gemm: $(tr '\n' ' ' < gpurun_out/ab/gemm_$v.$r.log)"
    fi
    if [ -z "$NO_GEMV" ]; then
      GGML_HIP_LIB=$lib timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu --no-prefill --no-exact --no-extra \
          > gpurun_out/ab/bench_$v.$r.log 2>&1 || { echo "bench $v rc=$?"; exit 1; }
      python - "$v" gpurun_out/ab/bench_$v.$r.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ps = r["roofline"]["per_shape"]
print(f"{sys.argv[1]:10s} decode", r["value"], r["roofline"]["frac"], " ".join(f"{k.split('->')[1]}={v['us']}" for k, v in ps.items()))
PY
    fi
  done
done
exit 0
