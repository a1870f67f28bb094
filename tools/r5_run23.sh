set -o pipefail
mkdir -p gpurun_out/r05
for r in 1 2; do
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-noepi,fast-nokq --out gpurun_out/r05/e2e_7b_ab$r.json > gpurun_out/r05/e2e_7b_ab$r.log 2>&1; echo "7b rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_7b_ab$r.json'))
for k,v in r.items():
    if k.startswith('offload'): print(k, v['decode_tok_s'], v['backend_host_ms_per_eval'], v['eager_launches_per_eval'])
"
done
timeout -k 10 300 python tools/e2e_llama.py --decode 512 --no-cpu --modes fast,fast-nokq --out gpurun_out/r05/e2e_7b_long.json > gpurun_out/r05/e2e_7b_long.log 2>&1; echo "long rc=$?"
python3 -c "
import json; r=json.load(open('gpurun_out/r05/e2e_7b_long.json'))
for k,v in r.items():
    if k.startswith('offload'): print('decode512', k, v['decode_tok_s'], v['backend_host_ms_per_eval'], v['eager_launches_per_eval'])
"
