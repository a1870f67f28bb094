set -o pipefail
mkdir -p gpurun_out/r05 gpurun_out/r05/hp3
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "launch_recorder or fusion or kq_fold" > gpurun_out/r05/thr_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r05/thr_tests.log
grep -q FAILED gpurun_out/r05/thr_tests.log && exit 1
timeout -k 10 600 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-thread,fast,fast-thread --hostprof gpurun_out/r05/hp3/h7b --out gpurun_out/r05/e2e_7b_thr2.json > gpurun_out/r05/e2e_7b_thr2.log 2>&1; echo "7b rc=$?"
gzip -f gpurun_out/r05/hp3/h7b.*
grep -E "^fast" gpurun_out/r05/e2e_7b_thr2.log | cut -c1-400
