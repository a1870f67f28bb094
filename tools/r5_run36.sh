set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_attn_decode.py > gpurun_out/r05/attn_t.tests.log 2>&1 && tail -1 gpurun_out/r05/attn_t.tests.log &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llama_ggjt.py -k "kq_fold or long_decode" > gpurun_out/r05/attn_t.model.log 2>&1 && tail -1 gpurun_out/r05/attn_t.model.log &&
timeout -k 10 300 python tools/attn_ab.py 200 > gpurun_out/r05/attn_ab_t.log 2>&1 && cat gpurun_out/r05/attn_ab_t.log
