#!/bin/bash
# HBM traffic of the decode GEMV from PMC counters: separate FETCH_SIZE and WRITE_SIZE passes
# (MI355X_MICROARCH.md §HBM: counters in their own run, kernel-trace only; no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c -d gpurun_out/pmc/$c -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prefill --no-extra > gpurun_out/pmc/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json; cat gpurun_out/pmc/summary.json
