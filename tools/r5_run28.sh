set -o pipefail
mkdir -p gpurun_out/r05
GGML_HIP_LIB=variants/libggml_hip_astamps.so timeout -k 10 200 python tools/attn_stamps.py > gpurun_out/r05/attn_stamps.txt 2>&1; echo "rc=$?"; cat gpurun_out/r05/attn_stamps.txt
