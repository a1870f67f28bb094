set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 500 python tools/e2e_llama.py --shape host --decode 64 --no-cpu --modes fast,exact --out gpurun_out/r05/e2e_host.json > gpurun_out/r05/e2e_host.log 2>&1
echo "e2e rc=$?"; tail -c 3000 gpurun_out/r05/e2e_host.json
