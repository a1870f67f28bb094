set -o pipefail
mkdir -p gpurun_out/r05
GGML_HIP_TRACE_NODES=1 timeout -k 10 300 python tools/e2e_llama.py --decode 24 --no-cpu --modes fast --out gpurun_out/r05/e2e_trace_nodes.json > gpurun_out/r05/e2e_trace_nodes.log 2>&1; echo "trace rc=$?"
python3 tools/node_gaps.py gpurun_out/r05/e2e_trace_nodes.log
gzip -f gpurun_out/r05/e2e_trace_nodes.log
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-noepi --out gpurun_out/r05/e2e_7b_xpn2.json > gpurun_out/r05/e2e_7b_xpn2.log 2>&1; echo "7b rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_7b_xpn2.json'))
for k,v in r.items():
    if k.startswith('offload'): print(k, v['decode_tok_s'], v['backend_host_ms_per_eval'], v['eager_launches_per_eval'])
"
