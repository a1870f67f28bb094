set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_gemv_epi.py tests/test_gpu_llama_ggjt.py -k "epilogue or norm_fold or fusion or glu or rope" > gpurun_out/r05/pxf_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/pxf_tests.log
grep -q -E "FAILED|[0-9]+ failed" gpurun_out/r05/pxf_tests.log && exit 1
for v in stamps stamps0; do
GGML_HIP_LIB=variants/libggml_hip_$v.so timeout -k 10 300 python tools/gemv_norm_stamps.py > gpurun_out/r05/gemv_norm_$v.txt 2>&1; echo "$v rc=$?"; cat gpurun_out/r05/gemv_norm_$v.txt
done
for r in 1 2; do
timeout -k 10 300 python tools/gemv_epi_ab.py 200 2 > gpurun_out/r05/gemv_epi_pxf1_$r.log 2>&1; echo "pxf1 rc=$?"; head -10 gpurun_out/r05/gemv_epi_pxf1_$r.log
GGML_HIP_LIB=variants/libggml_hip_pxf0.so timeout -k 10 300 python tools/gemv_epi_ab.py 200 2 > gpurun_out/r05/gemv_epi_pxf0_$r.log 2>&1; echo "pxf0 rc=$?"; head -10 gpurun_out/r05/gemv_epi_pxf0_$r.log
done
