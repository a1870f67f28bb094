#!/bin/bash
# round 2: register-ring GEMV, x-first (VAR 7) vs production (VAR 3): phase stamps + decode A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
for v in 3 15; do for km in "4096 4096" "11008 4096"; do
  set -- $km
  echo "VAR=$v K=$1 M=$2"
  XW=11 K=$1 M=$2 GGML_HIP_GEMV_VAR=$v GGML_HIP_GEMV_LDS=0 timeout -k 10 120 python tools/gemv_stamps.py || exit $?
done; done
for rep in 1 2; do for v in 3 15; do
  GGML_HIP_GEMV_VAR=$v timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu --no-prefill --no-exact > gpurun_out/r2/var_ab_$v.$rep.log 2>&1 || exit $?
  python3 - gpurun_out/r2/var_ab_$v.$rep.log $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ps={k:v["us"] for k,v in d["roofline"]["per_shape"].items()}
print("VAR",sys.argv[2],"tok/s",d["value"],"frac",d["roofline"]["frac"],ps,[ (c["config"][:10],c["tok_s"]) for c in d.get("other_configs",[])])
PY
done; done
