#!/bin/bash
# Interleaved A/B of whole-library variants on the LLaMA-7B decode headline (per-shape launch times):
#   LIBS="base xko1" ROUNDS=2 bash tools/r5_ab_decode.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu \
        --no-prefill --no-exact --no-extra > gpurun_out/ab/dec_$v.$r.log 2> gpurun_out/ab/dec_$v.$r.err || { echo "$v rc=$?"; tail -5 gpurun_out/ab/dec_$v.$r.err; exit 1; }
    python - "$v" gpurun_out/ab/dec_$v.$r.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ps = r["roofline"]["per_shape"]
print(f"{sys.argv[1]:8s} {r['value']} tok/s frac {r['roofline']['frac']} |", " ".join(f"{k.split('->')[1]}={v['us']}" for k, v in ps.items()), flush=True)
PY
  done
done
