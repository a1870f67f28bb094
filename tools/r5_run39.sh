# 128 x 128 k_gemm9 tile chosen per launch by rounds of CUs (auto) vs the round's base library: tests, per-shape
# kernel medians with the tile forced each way, then the bench prefill A/B.
set -o pipefail
O=gpurun_out/r05/wide2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gemm9 or gemm8 or sibling or image" > $O/tests.log 2>&1; echo "parity rc=$?"; tail -2 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_x9.py tests/test_gpu_llama_ggjt.py -k "x9 or x_image or prefill" > $O/tests2.log 2>&1; echo "model rc=$?"; tail -2 $O/tests2.log
for w in 0 1; do
  for shp in "4096 22016 512" "4096 4096 1024" "4096 12288 512" "4096 11008 1024" "11008 4096 1024" "4096 4096 2048"; do
    set -- $shp
    d=$O/p_w${w}_$1_$2_$3
    GGML_HIP_GEMM9_WIDE=$w K=$1 M=$2 N=$3 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gemm_one.py > $d.log 2>&1 || { echo "w$w $shp failed"; tail -3 $d.log; exit 1; }
    python3 - "w$w" "$shp" $d <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_gemm9" in r["Kernel_Name"]]
K, M, N = map(int, sys.argv[2].split())
med = statistics.median(t)
print(f"{sys.argv[1]:5s} K={K:5d} M={M:5d} N={N:4d}: k_gemm9 median {med:7.2f} us min {min(t):7.2f} (n={len(t)}) {2*K*M*N/med/1e6:6.0f} TOP/s", flush=True)
PY
  done
done
LIBS="base auto" ROUNDS=3 PREFILL=1 bash tools/r5_ab.sh
