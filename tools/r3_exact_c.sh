#!/bin/bash
# exact decode chunk length (GGML_HIP_EXACT_C 64 / 32): the bitwise exact-mode tests with 32, then the
# bench's exact_mode line for both, 2 interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3exc
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
GGML_HIP_EXACT_C=32 GGML_HIP_EXACT_S=${TEST_S:-2} timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_llama_ggjt.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -n 2 $O/t.log; case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for cs in ${CS:-64:2 32:2}; do
    c=${cs%:*}; sl=${cs#*:}
    GGML_HIP_EXACT_C=$c GGML_HIP_EXACT_S=$sl timeout -k 10 300 python bench.py --no-cpu --no-prefill --no-extra > $O/b$c.$r.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
    echo "EXACT_C $c slots $sl round $r: $(tail -n 1 $O/b$c.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["exact_mode"])')"
  done
done
