set -o pipefail
mkdir -p gpurun_out/r05
GGML_HIP_LIB=$PWD/variants/libggml_hip_g9ow.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm9 or gemm8_registered or prefill" > gpurun_out/r05/g9ow_tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/r05/g9ow_tests.log | tail -8
LIBS="base g9ow" bash tools/r5_g9ko.sh
LIBS="base g9ow" ROUNDS=2 PREFILL=1 bash tools/r5_ab.sh
