set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 500 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_gemv_epi.py tests/test_gpu_llama_ggjt.py tests/test_gpu_ggml_hook.py tests/test_gpu_f16_mul_mat.py > gpurun_out/r05/kq_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r05/kq_tests.log
grep -q FAILED gpurun_out/r05/kq_tests.log && exit 1
mkdir -p gpurun_out/r05/hp2 && timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-nokq,fast-thread --hostprof gpurun_out/r05/hp2/h7b --out gpurun_out/r05/e2e_7b_kq.json > gpurun_out/r05/e2e_7b_kq.log 2>&1; gzip -f gpurun_out/r05/hp2/h7b.*
echo "7b rc=$?"
GGML_HIP_GRAPH=2 GGML_HIP_TRACE_GRAPH=1 timeout -k 10 300 python tools/e2e_llama.py --shape host --decode 16 --no-cpu --modes fast-thread > gpurun_out/r05/e2e_thr_trace.log 2>&1
echo "trace rc=$?"
python3 - <<'PY'
import json, collections
r = json.load(open("gpurun_out/r05/e2e_7b_kq.json"))
for k, v in r.items():
    if k.startswith("offload"):
        print(k, v["decode_tok_s"], v.get("backend_host_ms_per_eval"), v.get("eager_launches_per_eval"), v.get("graph_per_eval"))
c = collections.Counter(l.split(" by ")[1].strip() for l in open("gpurun_out/r05/e2e_thr_trace.log") if l.startswith("rec_flush"))
print(c.most_common(20))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_e2e3 -o e2e -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast > gpurun_out/r05/prof_e2e3.log 2>&1
echo "prof rc=$?"
timeout -k 10 300 python tools/gemv_epi_ab.py 200 3 > gpurun_out/r05/gemv_epi_ab.log 2>&1; echo "epi_ab rc=$?"; cat gpurun_out/r05/gemv_epi_ab.log | head -12
