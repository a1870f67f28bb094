# Price a K split of the 128 x 128 tile before building it: the wide tile at half K with twice the rows has exactly
# the workgroup count and per-workgroup work of a 2-way K split (no hand-off), against the 128 x 64 tile at full K.
set -o pipefail
O=gpurun_out/r05/splitk; mkdir -p $O
for shp in "0 4096 4096 512" "1 2048 8192 512" "0 11008 4096 512" "1 5504 8192 512" "0 4096 12288 512" "1 2048 24576 512"; do
  set -- $shp
  d=$O/p_w$1_$2_$3_$4
  GGML_HIP_GEMM9_WIDE=$1 K=$2 M=$3 N=$4 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gemm_one.py > $d.log 2>&1 || exit 1
  python3 - "w$1" "$2 $3 $4" $d <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
g = [r for r in rows if "k_gemm9" in r["Kernel_Name"]]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in g]
print(f"{sys.argv[1]} K M N = {sys.argv[2]}: k_gemm9 median {statistics.median(t):7.2f} us (n={len(t)}, {len(set(r['Kernel_Name'][:25] for r in g))} kernel kinds)", flush=True)
PY
done
