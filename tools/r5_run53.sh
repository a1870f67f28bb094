# half tiles for single-round launches of at most half the CUs (GGML_HIP_GEMM9_HALF=2) vs the tail only (1)
set -o pipefail
O=gpurun_out/r05; mkdir -p $O
for r in 1 2; do for h in 1 2; do
  GGML_HIP_GEMM9_HALF=$h NS="96 128 192 256" timeout -k 10 400 python tools/g9_tile_sweep.py > $O/half_${h}_$r.jsonl 2> $O/half_${h}_$r.err || exit 1
done; done
GGML_HIP_GEMM9_HALF=2 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gemm9 or image or sibling" > $O/half2.tests.log 2>&1; tail -1 $O/half2.tests.log
