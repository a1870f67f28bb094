# Decode attention, short rows: every wave takes the softmax max / sum itself (no cross-wave reduction, no barrier
# after the KQ row) vs the shipped three-barrier softmax.  Bitwise tests on the new build, kernel A/B, e2e A/B.
set -o pipefail
O=gpurun_out/r05/redun; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_attn_decode.py > $O/t.log 2>&1 && tail -1 $O/t.log &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "kq_fold or long_decode or exact" > $O/m.log 2>&1 && tail -1 $O/m.log || exit 1
for v in base redun base redun; do
  GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 300 python tools/attn_ab.py 200 > $O/ab_$v.log 2>&1 || exit 1
  echo "== $v"; head -4 $O/ab_$v.log
done
for r in 1 2; do for v in base redun; do
  GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 300 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast --out $O/e2e_${v}_$r.json > $O/e2e_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json; r=json.load(open('$O/e2e_${v}_$r.json'))['offload_fast']; print('$v', r['decode_tok_s'], 'tok/s')"
done; done
