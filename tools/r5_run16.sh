set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast-thread,fast --out gpurun_out/r05/e2e_7b_thr3.json > gpurun_out/r05/e2e_7b_thr3.log 2>&1; echo "7b rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_7b_thr3.json'))
for k,v in r.items():
    if k.startswith('offload'): print(k, v['decode_tok_s'], v['backend_host_ms_per_eval'], v['eager_launches_per_eval'], v['eager_launch_host_ms_per_eval'], v['graph_per_eval'])
"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GGML_HIP_GRAPH=2 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_thr -o e2e -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast-thread > gpurun_out/r05/prof_thr.log 2>&1
echo "prof rc=$?"
