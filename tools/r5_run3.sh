set -o pipefail
mkdir -p gpurun_out/r05
GGML_HIP_LIB=$PWD/variants/libggml_hip_g9pf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm9 or gemm8_registered or prefill" > gpurun_out/r05/g9pf_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/g9pf_tests.log
LIBS="base g9pf" ROUNDS=3 PREFILL=1 bash tools/r5_ab.sh
