#!/bin/bash
# k_prep9_x: DPP row shifts vs __shfl field gathers (GGML_HIP_PREP9_DPP), interleaved on one box under
# rocprofv3 kernel traces; the gemm9 parity tests first (the x image feeds the bitwise gemm9 == gemm8 tests).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/prep9
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
step tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "gemm9 or image or sibling"
tail -1 $O/tests.log
for r in 1 2; do
  for d in 1 0; do
    GGML_HIP_PREP9_DPP=$d step prof_d${d}_r$r 300 rocprofv3 --kernel-trace --stats -d $O/prof_d${d}_r$r -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extra --no-exact
    python3 tools/trace_summary.py $(ls $O/prof_d${d}_r$r/*/run_kernel_trace.csv $O/prof_d${d}_r$r/run_kernel_trace.csv 2>/dev/null | head -1) > $O/ts_d${d}_r$r.txt 2>&1
    echo "dpp=$d round $r"; grep -E "prep9_x|gemm9" $O/ts_d${d}_r$r.txt
    grep -o '"prefill": {[^}]*' $O/prof_d${d}_r$r.log | cut -c1-120
  done
done
