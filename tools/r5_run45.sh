# x9 image stores: lane 0 of each 8-lane group gathers the block's fields and stores whole 16-byte pieces (st16)
# vs two dword stores per lane (base): bitwise tests on the new build, k_prep9_x medians, bench prefill A/B.
set -o pipefail
O=gpurun_out/r05/st16; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_x9.py tests/test_gpu_parity.py -k "x9 or gemm9 or prefill" > $O/t.log 2>&1 && tail -1 $O/t.log &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "x_image or prefill" > $O/m.log 2>&1 && tail -1 $O/m.log || exit 1
for r in 1 2; do for v in base st16; do
  for K in 4096 11008; do
    d=$O/p_${v}_${K}_$r
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so K=$K M=4096 N=512 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gemm_one.py > $d.log 2>&1 || exit 1
    python3 - "$v" "$K" $d <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "prep9_x" in r["Kernel_Name"]]
print(f"{sys.argv[1]:5s} K={sys.argv[2]:5s} N=512: k_prep9_x median {statistics.median(t):6.2f} us min {min(t):6.2f}", flush=True)
PY
  done
done; done
LIBS="base st16" ROUNDS=2 PREFILL=1 bash tools/r5_ab.sh
