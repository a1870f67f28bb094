# 128 x 128 k_gemm9 tile: stage hand-offs by LDS counters (GGML_HIP_GEMM9W_FLAGS=1) vs a barrier per stage (shipped)
set -o pipefail
O=gpurun_out/r05/flg; mkdir -p $O
GGML_HIP_GEMM9W_FLAGS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "wide or sibling_group or auto_tile" > $O/t1.log 2>&1; rc=$?; tail -1 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for f in 0 1; do
  for shp in "4096 22016 512" "4096 4096 1024" "11008 4096 1024" "4096 4096 2048"; do
    set -- $shp
    d=$O/p_f${f}_$1_$2_$3_$r
    GGML_HIP_GEMM9W_FLAGS=$f GGML_HIP_GEMM9_WIDE=1 K=$1 M=$2 N=$3 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gemm_one.py > $d.log 2>&1 || exit 1
    python3 - "f$f" "$shp" $d <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "k_gemm9" in r["Kernel_Name"]]
print(f"{sys.argv[1]} K M N = {sys.argv[2]}: k_gemm9w median {statistics.median(t):7.2f} us (n={len(t)})", flush=True)
PY
  done
done; done
for r in 1 2; do for f in 0 1; do
  GGML_HIP_GEMM9W_FLAGS=$f timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu --no-exact --no-extra > $O/b_f${f}_$r.log 2> $O/b_f${f}_$r.err || exit 1
  python3 -c "
import json; r=json.loads(open('$O/b_f${f}_$r.log').read().strip().splitlines()[-1]); print('f$f bench prefill', r['prefill']['TOPs'], 'TOP/s', r['prefill']['ms_per_layer'], 'ms/layer')"
done; done
