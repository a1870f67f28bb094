set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_attn_decode.py > gpurun_out/r05/attn_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/attn_tests.log
grep -q -E "FAILED|[0-9]+ failed" gpurun_out/r05/attn_tests.log && exit 1
timeout -k 10 300 python tools/attn_ab.py 200 > gpurun_out/r05/attn_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05/attn_ab.log
