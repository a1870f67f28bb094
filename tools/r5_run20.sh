set -o pipefail
mkdir -p gpurun_out/r05
for r in 1 2; do
for v in main nko1 nko2; do
if [ $v = main ]; then L=""; else L=variants/libggml_hip_$v.so; fi
GGML_HIP_LIB=$L timeout -k 10 300 python tools/gemv_epi_ab.py 200 2 > gpurun_out/r05/gemv_nko_${v}_$r.log 2>&1; echo "$v rc=$?"; head -10 gpurun_out/r05/gemv_nko_${v}_$r.log | grep -E "qkv|w1"
done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "kq_fold or long_decode" > gpurun_out/r05/kqu_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/kqu_tests.log
grep -q -E "FAILED|[0-9]+ failed" gpurun_out/r05/kqu_tests.log && exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_e2e4 -o e2e -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast > gpurun_out/r05/prof_e2e4.log 2>&1
echo "prof rc=$?"
