set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "epilogue or fusion or norm_fold or launch_recorder" > gpurun_out/r05/epi_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r05/epi_tests.log
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-noepi,fast-thread --out gpurun_out/r05/e2e_7b_epi.json > gpurun_out/r05/e2e_7b_epi.log 2>&1
echo "7b rc=$?"
python3 - <<'PY'
import json
r = json.load(open("gpurun_out/r05/e2e_7b_epi.json"))
for k, v in r.items():
    if k.startswith("offload"):
        print(k, v["decode_tok_s"], v.get("backend_host_ms_per_eval"), v.get("eager_launches_per_eval"))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/prof_e2e -o e2e -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast > gpurun_out/r05/prof_e2e.log 2>&1
echo "prof rc=$?"
find gpurun_out/r05/prof_e2e -name "*kernel_stats.csv" | head -2
