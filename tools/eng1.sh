set -o pipefail
mkdir -p gpurun_out/r06/eng1
export GGML_HIP_ENGINE_TIMEOUT_MS=1000
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_chain.py -k engine > gpurun_out/r06/eng1/tests.log 2>&1; rc=$?; tail -15 gpurun_out/r06/eng1/tests.log; echo "tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-exact --no-prefill > gpurun_out/r06/eng1/bench.log 2>&1; rc=$?; tail -c 3000 gpurun_out/r06/eng1/bench.log; echo "bench rc=$rc"
