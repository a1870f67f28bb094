set -o pipefail
mkdir -p gpurun_out/r05/spin2
for r in 1 2 3 4; do
for v in eager thr; do
case $v in eager) M=fast;; thr) M=fast-thread;; esac
timeout -k 10 300 python tools/e2e_llama.py --decode 128 --no-cpu --modes $M --out gpurun_out/r05/spin2/$v.$r.json > gpurun_out/r05/spin2/$v.$r.log 2>&1 || exit 1
python3 -c "
import json; r=json.load(open('gpurun_out/r05/spin2/$v.$r.json'))
print('$v', $r, [round(v['decode_tok_s'], 1) for k, v in r.items() if k.startswith('offload')])
"
done
done
