set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 500 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_llama_ggjt.py tests/test_gpu_ggml_hook.py > gpurun_out/r05/epi2_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r05/epi2_tests.log
[ -n "$(grep -c FAILED gpurun_out/r05/epi2_tests.log | grep -v '^0$')" ] && exit 1
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-noepi,fast-thread --out gpurun_out/r05/e2e_7b_epi2.json > gpurun_out/r05/e2e_7b_epi2.log 2>&1
echo "7b rc=$?"
GGML_HIP_GEMV_GLU_MAP=0 timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast --out gpurun_out/r05/e2e_7b_epi2_map0.json > gpurun_out/r05/e2e_7b_epi2_map0.log 2>&1
echo "7b map0 rc=$?"
python3 - <<'PY'
import json
for f in ("gpurun_out/r05/e2e_7b_epi2.json", "gpurun_out/r05/e2e_7b_epi2_map0.json"):
    r = json.load(open(f))
    for k, v in r.items():
        if k.startswith("offload"):
            print(f.split("/")[-1], k, v["decode_tok_s"], v.get("backend_host_ms_per_eval"), v.get("eager_launches_per_eval"))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_e2e2 -o e2e -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast > gpurun_out/r05/prof_e2e2.log 2>&1
echo "prof rc=$?"
