# mixed 128x128 + 128x64 launches on by default: tests, then bench prefill with GGML_HIP_GEMM9_MIXED=0 / 1
set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gemm9 or gemm8 or wide or auto_tile or sibling or image" > $O/mixed.tests.log 2>&1; rc=$?; tail -1 $O/mixed.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_x9.py tests/test_gpu_llama_ggjt.py -k "x9 or x_image or prefill" > $O/mixed.tests2.log 2>&1; rc=$?; tail -1 $O/mixed.tests2.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for m in 0 1; do
  GGML_HIP_GEMM9_MIXED=$m timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu --no-exact --no-extra > $O/bm_${m}_$r.log 2> $O/bm_${m}_$r.err || exit 1
  python3 -c "
import json; r=json.loads(open('$O/bm_${m}_$r.log').read().strip().splitlines()[-1]); print('mixed=$m bench prefill', r['prefill']['TOPs'], 'TOP/s', r['prefill']['ms_per_layer'], 'ms/layer')"
done; done
