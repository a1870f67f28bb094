# k_prep9_x knockouts (timing only): pko1 no loads, pko2 loads + encode without stores, pko3 loads only
set -o pipefail
O=gpurun_out/r05/pko; mkdir -p $O
for r in 1 2; do for v in base pko1 pko2 pko3; do
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
