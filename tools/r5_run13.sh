set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-thread --out gpurun_out/r05/e2e_7b_thr.json > gpurun_out/r05/e2e_7b_thr.log 2>&1
echo "7b rc=$?"
GGML_HIP_GRAPH=2 GGML_HIP_TRACE_GRAPH=1 timeout -k 10 300 python tools/e2e_llama.py --shape host --decode 16 --no-cpu --modes fast-thread > gpurun_out/r05/e2e_thr_trace.log 2>&1
echo "trace rc=$?"
python3 - <<'PY'
import json, collections
r = json.load(open("gpurun_out/r05/e2e_7b_thr.json"))
for k, v in r.items():
    if k.startswith("offload"):
        print(k, v["decode_tok_s"], v.get("backend_host_ms_per_eval"), v.get("eager_launches_per_eval"), v.get("graph_per_eval"))
c = collections.Counter(l.split(" by ")[1].strip() for l in open("gpurun_out/r05/e2e_thr_trace.log") if l.startswith("rec_flush"))
print(c.most_common(20))
PY
