set -o pipefail
mkdir -p gpurun_out/r05/pf
for r in 1 2; do
for mb in 0 4 8 16 64; do
timeout -k 10 300 python bench.py --no-prefill --no-cpu --no-extra --no-exact --prefetch-mb $mb > gpurun_out/r05/pf/b$mb.$r.log 2> gpurun_out/r05/pf/b$mb.$r.err || { echo "mb $mb failed"; tail -5 gpurun_out/r05/pf/b$mb.$r.err; exit 1; }
python3 -c "
import json; r=json.loads(open('gpurun_out/r05/pf/b$mb.$r.log').read().strip().splitlines()[-1])
ps = r['roofline']['per_shape']
print('pf', $mb, 'MB round', $r, r['value'], 'tok/s', r['config']['activations_finite'], {k: v['us'] for k, v in ps.items()})
"
done
done
