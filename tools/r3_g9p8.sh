#!/bin/bash
# k_gemm9 variant A/B (GGML_HIP_GEMM9_VAR VB vs VA; default 17 = the K = 8 scale MFMA vs 1): bitwise
# gemm9 tests under VAR VB, then kernel medians per LLaMA-7B shape (tools/r3_g9var.sh) and the bench
# prefill, 2 interleaved rounds on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g9p8_${VB:-17}
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
GGML_HIP_GEMM9_VAR=${VB:-17} step tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "gemm9 or image or sibling"
tail -1 $O/tests.log
grep -q " passed" $O/tests.log && ! grep -q "failed" $O/tests.log || exit 3
VARS="${VA:-1} ${VB:-17}" bash tools/r3_g9var.sh
for r in 1 2; do
  for v in ${VB:-17} ${VA:-1}; do
    GGML_HIP_GEMM9_VAR=$v step bench_v${v}_r$r 200 python bench.py --no-cpu --no-extra --no-exact --steps 5 --warmup 2
    python3 -c "import json; d=json.loads(open('$O/bench_v${v}_r$r.log').read().strip().splitlines()[-1]); p=d['prefill']; print('VAR $v round $r: prefill ms/layer', p['ms_per_layer'], 'TOP/s', p['TOPs'])"
  done
done
