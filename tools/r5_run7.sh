set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "gemm9 or gemm8 or prefill or image" > gpurun_out/r05/half_tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/r05/half_tests.log | tail -5
LIBS="base half" bash tools/r5_g9ko.sh
LIBS="base half" ROUNDS=2 PREFILL=1 bash tools/r5_ab.sh
