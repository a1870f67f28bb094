#!/bin/bash
# counters of the k_gemm9 compute-only knockout vs k_gemm8's (4096 x 4096 x 512), one pass per set
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3g9p
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
i=0
IFS=, read -ra VDS <<< "${VDS:-11 93,9 83,11 0}"
for vd in "${VDS[@]}"; do
  set -- $vd
  for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    GGML_HIP_GEMM_V=$1 GGML_HIP_GEMM_DIAG=$2 timeout -s KILL 90 rocprofv3 --pmc $c -d $O/p$i -o run --output-format csv -- python3 tools/gemm_stamps.py > $O/p$i.log 2>&1
    rc=$?; case $rc in 0) ;; *) echo "rc=$rc at $vd / $c"; exit $rc;; esac
    python3 - "$O/p$i" "$1 $2" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gemm" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("V/DIAG", sys.argv[2], " ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(tot.items())))
PY
  done
done
