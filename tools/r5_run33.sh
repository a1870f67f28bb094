set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 480 python bench.py --no-prefill --no-cpu --no-exact > gpurun_out/r05/bench_falcon.log 2> gpurun_out/r05/bench_falcon.err; echo "bench rc=$?"
python3 -c "
import json; r=json.loads(open('gpurun_out/r05/bench_falcon.log').read().strip().splitlines()[-1])
print(r['value'], r['roofline']['frac'])
for c in r['other_configs']: print(c)
"
