set -o pipefail
mkdir -p gpurun_out/r05
for v in 15 3; do
GGML_HIP_GEMV_VAR=$v GGML_HIP_LIB=variants/libggml_hip_stamps.so timeout -k 10 300 python tools/gemv_norm_stamps.py > gpurun_out/r05/gemv_norm_stamps_v$v.txt 2>&1; echo "stamps v$v rc=$?"
cat gpurun_out/r05/gemv_norm_stamps_v$v.txt
done
for v in 15 3; do
GGML_HIP_GEMV_VAR=$v timeout -k 10 300 python tools/gemv_epi_ab.py 200 2 > gpurun_out/r05/gemv_epi_ab_v$v.log 2>&1; echo "ab v$v rc=$?"; head -10 gpurun_out/r05/gemv_epi_ab_v$v.log
done
