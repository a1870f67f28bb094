#!/bin/bash
# e2e decode tok/s of the full-offload path under several environment settings (one e2e run each):
#   ENVS="X=1 GGML_HIP_GRAPH=0" DECODE=128 bash tools/e2e_env_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in $ENVS; do
  env $(echo "$e" | tr ',' ' ') timeout -k 10 300 python tools/e2e_llama.py --no-cpu --modes fast --decode ${DECODE:-128} \
      > gpurun_out/e2e_env.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/e2e_env.log; exit 1; }
  python - "$e" <<'PY'
import json, sys
r = json.loads(open("gpurun_out/e2e_env.log").read().strip().splitlines()[-1])["offload_fast"]
print(f"{sys.argv[1]:40s}", r["decode_tok_s"], r["backend_host_ms_per_eval"], r["graph_per_eval"], r["backend_per_op"].get("mul"))
PY
done
