set -o pipefail
O=gpurun_out/r05; mkdir -p $O
for r in 1 2; do for m in 0 1; do
  GGML_HIP_GEMM9_MIXED=$m timeout -k 10 300 python tools/g9_mixed_check.py > $O/mixed_${m}_$r.jsonl 2> $O/mixed_${m}_$r.err || exit 1
done; done
cat $O/mixed_1_1.jsonl
