# bench prefill, mixed k_gemm9 launches off / on, 5 interleaved rounds
set -o pipefail
O=gpurun_out/r05; mkdir -p $O
for r in 1 2 3 4 5; do for m in 0 1; do
  GGML_HIP_GEMM9_MIXED=$m timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --no-exact --no-extra > $O/bm2_${m}_$r.log 2> $O/bm2_${m}_$r.err || exit 1
  python3 -c "
import json; r=json.loads(open('$O/bm2_${m}_$r.log').read().strip().splitlines()[-1]); print('mixed=$m', r['prefill']['TOPs'], 'TOP/s', r['prefill']['ms_per_layer'], 'ms/layer', r['value'], 'tok/s')"
done; done
