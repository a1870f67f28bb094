#!/bin/bash
# decode per-layer time when the weight stack fits the Infinity Cache (L = 1, 2) vs HBM (32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
for L in ${LAYERS:-1 2 32}; do
  timeout -k 10 120 python bench.py --layers $L --steps 200 --warmup 20 --no-cpu --no-prefill --no-exact --no-extra > gpurun_out/r2/mall_L$L.log 2>&1 || exit 1
  python - $L <<'PY'
import json, sys
L = int(sys.argv[1])
d = json.loads(open(f"gpurun_out/r2/mall_L{L}.log").read().strip().splitlines()[-1])
print(L, d["ms_per_step"], round(d["ms_per_step"] / L * 1000, 2), "us/layer",
      {k.split("->")[1]: v["us"] for k, v in d["roofline"]["per_shape"].items()})
PY
done
