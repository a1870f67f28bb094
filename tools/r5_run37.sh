# x9 encoder by byte-table lookups (tab) vs base: bitwise tests on the new library, then interleaved A/B
set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x9.py tests/test_gpu_parity.py -k "x9 or gemm9 or prefill" > $O/tab.tests.log 2>&1 && tail -1 $O/tab.tests.log &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "x_image" > $O/tab.model.log 2>&1 && tail -1 $O/tab.model.log &&
for v in base tab; do
  for K in 4096 11008; do
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so K=$K timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/tabprof_${v}_$K -o run --output-format csv -- python3 tools/gemm_one.py > $O/tabprof_${v}_$K.log 2>&1 || exit 1
    grep -h "prep9_x" $(find $O/tabprof_${v}_$K -name "*kernel_stats.csv") | cut -d, -f1-4 | sed "s/^/$v K=$K /"
  done
done &&
LIBS="base tab" ROUNDS=3 PREFILL=1 bash tools/r5_ab.sh
