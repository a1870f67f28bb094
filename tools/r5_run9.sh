set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python tools/e2e_llama.py --shape host --decode 64 --no-cpu --modes fast,fast-thread,fast-graph --out gpurun_out/r05/e2e_host_modes.json > gpurun_out/r05/e2e_host_modes.log 2>&1
echo "host rc=$?"
timeout -k 10 700 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-thread,fast-graph,exact --out gpurun_out/r05/e2e_7b_modes.json > gpurun_out/r05/e2e_7b_modes.log 2>&1
echo "7b rc=$?"
python3 - <<'PY'
import json
for f in ("gpurun_out/r05/e2e_host_modes.json", "gpurun_out/r05/e2e_7b_modes.json"):
    try:
        r = json.load(open(f))
    except Exception as e:
        print(f, e); continue
    for k, v in r.items():
        if k.startswith("offload"):
            print(f.split("/")[-1], k, v["decode_tok_s"], v.get("backend_host_ms_per_eval"), v.get("eager_launch_host_ms_per_eval"), v.get("graph_per_eval"))
PY
