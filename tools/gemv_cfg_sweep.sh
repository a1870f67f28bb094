#!/bin/bash
# GEMV (waves per WG : ring depth : WGs per CU) sweep; prints decode tok/s and per-shape launch us
# from bench.py's event-timed graph chains.  CFGS="16:2:2 8:4:1 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
export PYTHONUNBUFFERED=1
for c in ${CFGS:-16:2:2 16:4:2 16:4:1 8:2:2 8:4:1 8:4:2 8:4:4 4:4:2 4:8:1 4:8:2 4:4:4}; do
  IFS=: read w d g <<< "$c"
  GGML_HIP_GEMV_WAVES=$w GGML_HIP_GEMV_DEPTH=$d GGML_HIP_GEMV_WG_PER_CU=$g timeout -k 10 240 \
    python bench.py --steps 20 --warmup 3 --no-cpu --no-prefill > gpurun_out/cfg/$w-$d-$g.log 2>&1
  rc=$?
  python - "$c" gpurun_out/cfg/$w-$d-$g.log <<'PY'
import json, sys
try:
    r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    ps = r["roofline"]["per_shape"]
    print(sys.argv[1], r["value"], r["roofline"]["frac"], " ".join(f"{k.split('->')[1]}={v['us']}" for k, v in ps.items()))
except Exception as e:
    print(sys.argv[1], "parse failed", e)
PY
  case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
done
exit 0
