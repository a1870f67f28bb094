#!/bin/bash
# SQ counters of the prefill GEMM (one counter set per rocprofv3 pass, kernel-trace implied).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gpmc
export TMPDIR=/tmp PYTHONUNBUFFERED=1 GGML_HIP_GEMM_DIAG=0
i=0
# SETS: counter sets separated by '|' (one rocprofv3 pass each)
IFS='|' read -ra sets <<< "${SETS:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA|SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS}"
for c in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/gpmc/p$i -o run --output-format csv -- python3 tools/gemm_stamps.py > gpurun_out/gpmc/p$i.log 2>&1
  rc=$?; echo "set $i ($c) rc=$rc"; case $rc in 0) ;; *) tail -5 gpurun_out/gpmc/p$i.log; exit $rc;; esac
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(list)
for f in glob.glob("gpurun_out/gpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(tot.items()):
    print(f"{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
PY
