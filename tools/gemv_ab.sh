#!/bin/bash
# Interleaved A/B of GEMV variants in one box: ROUNDS x each "NAME=ENV1,ENV2" spec, decode bench only.
#   SPECS="base=GGML_HIP_GEMV_DEPTH=1 glb=GGML_HIP_GEMV_VAR=1,GGML_HIP_GEMV_DEPTH=1" bash tools/gemv_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in $SPECS; do
    name=${spec%%=*}; envs=${spec#*=}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu --no-prefill --no-exact --no-extra \
        > gpurun_out/ab/$name.$r.log 2>&1
    rc=$?
    python - "$name" gpurun_out/ab/$name.$r.log <<'PY'
import json, sys
try:
    r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    ps = r["roofline"]["per_shape"]
    print(f"{sys.argv[1]:10s}", r["value"], r["roofline"]["frac"], " ".join(f"{k.split('->')[1]}={v['us']}" for k, v in ps.items()))
except Exception as e:
    print(sys.argv[1], "parse failed", e)
PY
    [ $rc = 0 ] || { echo "rc=$rc"; exit $rc; }
  done
done
exit 0
