set -o pipefail
mkdir -p gpurun_out/r05/hp
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast --hostprof gpurun_out/r05/hp/h7b --out gpurun_out/r05/e2e_7b_hp.json > gpurun_out/r05/e2e_7b_hp.log 2>&1
echo "7b rc=$?"
timeout -k 10 300 python tools/e2e_llama.py --shape host --decode 128 --no-cpu --modes fast --hostprof gpurun_out/r05/hp/hhost --out gpurun_out/r05/e2e_host_hp.json > gpurun_out/r05/e2e_host_hp.log 2>&1
echo "host rc=$?"
gzip -f gpurun_out/r05/hp/h7b.fast gpurun_out/r05/hp/hhost.fast && ls -la gpurun_out/r05/hp
