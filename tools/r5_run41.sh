# k_prep9_x workgroup size: 4 waves (256 threads, 2,048 workgroups at K = 4096, N = 512) vs 16 waves (1,024 threads)
set -o pipefail
O=gpurun_out/r05/prep; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x9.py > $O/t4.log 2>&1 && tail -1 $O/t4.log &&
GGML_HIP_PREP9_WAVES=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x9.py > $O/t16.log 2>&1 && tail -1 $O/t16.log || exit 1
for r in 1 2; do
for w in 4 16; do
  for K in 4096 11008; do
    d=$O/p_w${w}_${K}_$r
    GGML_HIP_PREP9_WAVES=$w K=$K M=4096 N=512 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/gemm_one.py > $d.log 2>&1 || exit 1
    python3 - "w$w" "$K" $d <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[3] + "/**/*kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "prep9_x" in r["Kernel_Name"]]
print(f"{sys.argv[1]:4s} K={sys.argv[2]:5s} N=512: k_prep9_x median {statistics.median(t):6.2f} us min {min(t):6.2f} (n={len(t)})", flush=True)
PY
  done
done
done
for r in 1 2; do for w in 4 16; do
GGML_HIP_PREP9_WAVES=$w timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu --no-exact --no-extra > $O/b_w${w}_$r.log 2> $O/b_w${w}_$r.err || exit 1
python3 -c "
import json,sys; r=json.loads(open('$O/b_w${w}_$r.log').read().strip().splitlines()[-1]); print('w$w', r['prefill']['TOPs'], 'TOP/s', r['prefill']['ms_per_layer'], 'ms/layer')"
done; done
