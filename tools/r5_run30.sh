set -o pipefail
mkdir -p gpurun_out/r05
for r in 1 2; do
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-thread --out gpurun_out/r05/e2e_7b_spin$r.json > gpurun_out/r05/e2e_7b_spin$r.log 2>&1; echo "7b rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_7b_spin$r.json'))
for k,v in r.items():
    if k.startswith('offload'): print(k, v['decode_tok_s'], v['backend_host_ms_per_eval'], v['eager_launch_host_ms_per_eval'], v['graph_per_eval']['runs'], v['graph_per_eval']['submit_ms'])
"
done
GGML_HIP_LAUNCHER_SPIN_US=1000000 timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast-thread --out gpurun_out/r05/e2e_7b_spinlong.json > gpurun_out/r05/e2e_7b_spinlong.log 2>&1; echo "7b rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_7b_spinlong.json'))
for k,v in r.items():
    if k.startswith('offload'): print('spin1s', k, v['decode_tok_s'], v['backend_host_ms_per_eval'])
"
