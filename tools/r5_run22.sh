set -o pipefail
mkdir -p gpurun_out/r05
for v in main kqu2 kqu8; do
if [ $v = main ]; then L=""; else L=variants/libggml_hip_$v.so; fi
GGML_HIP_LIB=$L timeout -k 10 300 python tools/attn_ab.py 200 > gpurun_out/r05/attn_ab_$v.log 2>&1; echo "$v rc=$?"; cat gpurun_out/r05/attn_ab_$v.log
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "long_decode or kq_fold" tests/test_gpu_attn_decode.py > gpurun_out/r05/kqmax_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/kqmax_tests.log
