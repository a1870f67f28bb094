#!/bin/bash
# Round-5 evidence pass on one MI355X: GPU tests, smoke, bench line, rocprofv3 kernel stats of the bench,
# decode-GEMV HBM traffic (PMC), prefill-GEMM counters.  Every GPU step has its own time limit; the
# script stops at the first step that faults, aborts or times out.  SKIP_TESTS=1 skips tests + smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {   # step <name> <seconds> <cmd...>  (counter passes: SIGKILL at the limit)
  local name=$1 t=$2; shift 2
  case $name in gpmc*|pmc_*) timeout -s KILL $t "$@" > $O/$name.log 2>&1;; *) timeout -k 10 $t "$@" > $O/$name.log 2>&1;; esac
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
# PART=tests | bench | e2e (one gpurun call each; default: all)
PART=${PART:-all}
if [ $PART = all -o $PART = tests ]; then
  step gputest 900 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread
  tail -3 $O/gputest.log
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ $PART = all -o $PART = bench ]; then
step bench 480 python bench.py
tail -1 $O/bench.log | cut -c1-300
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extra
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c -d $O/pmc/$c -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prefill --no-extra --no-exact
done
python3 tools/pmc_summary.py $O/pmc > $O/gemv_pmc_traffic.json
i=0
IFS='|' read -ra sets <<< "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA|SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS|FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE SQ_INSTS_SALU"
for c in "${sets[@]}"; do
  i=$((i+1))
  step gpmc$i 60 rocprofv3 --pmc $c -d $O/gpmc/p$i -o run --output-format csv -- python3 tools/gemm_one.py
done
python3 - <<'PY' > $O/gemm9_pmc.txt
import csv, glob, collections
tot = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r05f/gpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_gemm9" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("k_gemm9_q4_0 (registered fp6 image, tools/gemm_one.py), K=M=4096, N=512; mean per dispatch")
for k, v in sorted(tot.items()):
    print(f"{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
g = {k: sum(v) / len(v) for k, v in tot.items()}
if "GRBM_GUI_ACTIVE" in g and "SQ_VALU_MFMA_BUSY_CYCLES" in g:
    cyc = g["GRBM_GUI_ACTIVE"] / 8
    print(f"derived: MFMA busy {g['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f} of {cyc:.0f} cycles; "
          f"HBM read {2 * g.get('FETCH_SIZE', 0) * 1024 / 1e6:.1f} MB (2 x FETCH_SIZE, gfx950 half count); "
          f"write {g.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f} MB; VALU per MFMA {g.get('SQ_INSTS_VALU', 0) / max(1, g.get('SQ_INSTS_MFMA', 1)):.1f}; "
          f"WAIT_INST_ANY / WAVE_CYCLES {g.get('SQ_WAIT_INST_ANY', 0) / max(1, g.get('SQ_WAVE_CYCLES', 1)):.3f}")
PY
cat $O/gemm9_pmc.txt
fi
if [ $PART = all -o $PART = e2e ]; then
# the hook path end to end: the reference llama.cpp at full offload (LLaMA-7B shape), fast / exact, with a kernel trace
step e2e 700 python tools/e2e_llama.py --decode 128 --modes fast,exact --out $O/e2e_7b.json
step e2e_prof 600 rocprofv3 --kernel-trace --stats -d $O/prof_e2e -o e2e --output-format csv -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast
fi
