# The larger k_gemm9 tile (verdict r4 item 3): 128 x 128 per workgroup (GEMM9_WIDE) vs the shipped 128 x 64 with
# its K split, each with knockouts (GEMM9_KO 1 compute only, 2 no x DMA, 3 no weight DMA); rocprofv3 kernel
# medians over tools/gemm_one.py per shape, then the bench prefill line for base vs wide.
set -o pipefail
O=gpurun_out/r05/wide; mkdir -p $O
GGML_HIP_LIB=$PWD/variants/libggml_hip_wide.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "per_call_image or registered_image or sibling_group_one_launch or vs_oracle_edges" > $O/wide.tests.log 2>&1; echo "wide tests rc=$?"; tail -3 $O/wide.tests.log
for v in base wide ko1 wko1 ko2 wko2 ko3 wko3; do
  for shp in "4096 4096 512" "4096 4096 1024" "4096 11008 512" "11008 4096 512" "4096 12288 512"; do
    set -- $shp
    d=$O/p_${v}_$1_$2_$3
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so K=$1 M=$2 N=$3 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gemm_one.py > $d.log 2>&1 || { echo "$v $shp failed"; tail -3 $d.log; exit 1; }
    python3 - "$v" "$shp" $d <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_gemm9" in r["Kernel_Name"]]
K, M, N = map(int, sys.argv[2].split())
med = statistics.median(t)
print(f"{sys.argv[1]:5s} K={K:5d} M={M:5d} N={N:4d}: k_gemm9 median {med:7.2f} us min {min(t):7.2f} (n={len(t)}) {2*K*M*N/med/1e6:6.0f} TOP/s", flush=True)
PY
  done
done
LIBS="base wide" ROUNDS=2 PREFILL=1 bash tools/r5_ab.sh
