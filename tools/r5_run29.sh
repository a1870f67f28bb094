set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_attn_decode.py > gpurun_out/r05/attn2_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/attn2_tests.log
grep -q -E "FAILED|[0-9]+ failed" gpurun_out/r05/attn2_tests.log && exit 1
GGML_HIP_LIB=variants/libggml_hip_astamps.so timeout -k 10 200 python tools/attn_stamps.py > gpurun_out/r05/attn_stamps2.txt 2>&1; echo "rc=$?"; cat gpurun_out/r05/attn_stamps2.txt
timeout -k 10 300 python tools/attn_ab.py 200 > gpurun_out/r05/attn_ab2.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05/attn_ab2.log
