#!/bin/bash
# k_gemm9 sibling-group launch + XCD-aware tile order: parity tests, then an interleaved bench A/B of the
# prefill (GGML_HIP_GEMM9_XCD, GGML_HIP_GEMM9_GROUP), then a rocprofv3 kernel trace of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g9grp
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {   # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
if [ -z "$SKIP_TESTS" ]; then
  step tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "gemm9 or sibling or image or gemm8"
  tail -2 $O/tests.log
fi
for r in 1 2; do
  for cfg in "1 1" "0 0" "1 0" "0 1"; do
    set -- $cfg
    GGML_HIP_GEMM9_XCD=$1 GGML_HIP_GEMM9_GROUP=$2 step "bench_x$1_g$2_r$r" 200 python bench.py --no-cpu --no-extra --no-exact --steps 5 --warmup 2
    python3 -c "import json,sys; d=json.loads(open('$O/bench_x$1_g$2_r$r.log').read().strip().splitlines()[-1]); p=d['prefill']; print('xcd=$1 group=$2 round $r: prefill ms/layer', p['ms_per_layer'], 'TOP/s', p['TOPs'])"
  done
done
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extra --no-exact
python3 tools/trace_summary.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) > $O/trace_summary.txt 2>&1
grep -E "gemm9|prep9" $O/trace_summary.txt
