#!/bin/bash
# k_gemm9 (fp6 block sums) vs k_gemm8 (i8): the prefill-GEMM parity tests, then per-call-image kernel
# medians (GGML_HIP_GEMM_V 9 = gemm8, 11 = gemm9), 2 interleaved rounds, rocprofv3 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3g9
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ggml_hook.py -m gpu -x -q -k "gemm or prefill" --timeout 200 --timeout-method thread > $O/t.log 2>&1
  rc=$?; tail -3 $O/t.log; case $rc in 0) ;; *) exit $rc;; esac
fi
for r in 1 2; do
  for v in ${VERS:-9 11}; do
    GGML_HIP_GEMM_V=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $O/v$v.$r -o run --output-format csv -- python3 tools/gemm_shapes.py > $O/v$v.$r.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
    echo "version $v round $r"; python3 tools/kt_median.py $O/v$v.$r k_gemm; python3 tools/kt_median.py $O/v$v.$r prep
  done
done
