set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python tools/e2e_llama.py --shape host --decode 128 --no-cpu --modes fast,fast-thread,fast,fast-thread --out gpurun_out/r05/e2e_host_thr.json > gpurun_out/r05/e2e_host_thr.log 2>&1; echo "host rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_host_thr.json'))
for k,v in r.items():
    if k.startswith('offload'): print(k, v['decode_tok_s'], v['backend_host_ms_per_eval'], v['eager_launches_per_eval'], v['eager_launch_host_ms_per_eval'], v['graph_per_eval'])
"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GGML_HIP_GRAPH=2 timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d gpurun_out/r05/prof_thr_api -o e2e -- python3 tools/e2e_llama.py --decode 32 --no-cpu --modes fast-thread > gpurun_out/r05/prof_thr_api.log 2>&1
echo "prof rc=$?"
ls -la gpurun_out/r05/prof_thr_api/
