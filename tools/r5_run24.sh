set -o pipefail
mkdir -p gpurun_out/r05
for r in 1 2; do
for v in main xpn2 xpn1; do
for var in 15 3; do
if [ $v = main ]; then L=""; else L=variants/libggml_hip_$v.so; fi
GGML_HIP_GEMV_VAR=$var GGML_HIP_LIB=$L timeout -k 10 300 python tools/gemv_epi_ab.py 200 2 > gpurun_out/r05/gemv_xpn_${v}_v${var}_$r.log 2>&1; echo "$v var$var rc=$?"; head -10 gpurun_out/r05/gemv_xpn_${v}_v${var}_$r.log | grep -E "norm"
done
done
done
