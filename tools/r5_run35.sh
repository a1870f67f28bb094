set -o pipefail
mkdir -p gpurun_out/r05
for v in main at512 at256; do
if [ $v = main ]; then L=""; else L=variants/libggml_hip_$v.so; fi
GGML_HIP_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_attn_decode.py > gpurun_out/r05/attn_$v.tests.log 2>&1; echo "$v tests rc=$?"; tail -1 gpurun_out/r05/attn_$v.tests.log
GGML_HIP_LIB=$L timeout -k 10 300 python tools/attn_ab.py 200 > gpurun_out/r05/attn_ab_$v.log 2>&1; echo "$v ab rc=$?"; cat gpurun_out/r05/attn_ab_$v.log
done
