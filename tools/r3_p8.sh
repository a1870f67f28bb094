cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/p8
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ggml_hook.py -m gpu -x -q -k "gemm8 or prefill or q8_0" --timeout 120 --timeout-method thread > gpurun_out/p8/t.log 2>&1 && tail -2 gpurun_out/p8/t.log &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p8/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra --no-exact > gpurun_out/p8/b.log 2>&1 && python3 tools/trace_summary.py gpurun_out/p8/prof/run_kernel_trace.csv | grep -E "prep8|gemm8" && tail -1 gpurun_out/p8/b.log | cut -c1-200
