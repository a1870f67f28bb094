#!/bin/bash
# The one GPU job runner (replaces the round-4/5 one-off scripts; their history is in git).
#   PARTS="tests smoke bench prof pmc gpmc e2e e2e_variant" O=gpurun_out/r06 bash tools/run.sh
# Every GPU step runs under its own time limit; a fault, abort or timeout (rc 124/134/137/139 or any
# rc >= 2 of a step that must pass) ends the script there: no further GPU step in the same call.
# (aql needs tools/aql_dispatch_cost + tools/aql_kernel.hsaco, built by the hipcc lines in tools/aql_dispatch_cost.hip.)
# Extra arguments per part: BENCH_ARGS (bench, prof), E2E_ARGS (e2e), VARIANT (e2e_variant: a
# tools/build_variant.sh name under variants/, default base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/r06}
mkdir -p "$O"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
step() {   # step <name> <seconds> <cmd...>; counter passes get SIGKILL at the limit (rocprofv3 --pmc hangs on SIGTERM)
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  case $name in pmc_*|gpmc_*) timeout -s KILL "$t" "$@" > "$O/$name.log" 2>&1;;
                *) timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1;; esac
  local rc=$?
  echo "=== $name rc=$rc"
  case $rc in 0) return 0;; 1) tail -5 "$O/$name.log"; return 0;; *) tail -20 "$O/$name.log"; exit $rc;; esac
}
has() { [[ " ${PARTS:-tests smoke bench prof} " == *" $1 "* ]]; }

if has tests; then
  step gputest 1100 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread ${TEST_ARGS:-}
  grep -E "passed|failed" "$O/gputest.log" | tail -1
fi
has smoke && step smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
if has bench; then
  step bench 480 python bench.py ${BENCH_ARGS:-}
  tail -1 "$O/bench.log" | cut -c1-400
fi
if has prof; then    # the bench's own timed replays under the kernel tracer
  step prof 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-exact --no-roofline-replays --no-aql ${BENCH_ARGS:-}
  tail -1 "$O/prof.log" | cut -c1-300
  python3 tools/trace_steps.py "$O/prof" "$O/prof.log" > "$O/step_spans.json" || true
fi
if has final; then   # round-end evidence: the traced run first, installed under profiles/ (on the box), then the
  # bench, whose roofline.rocprof_check reads those files: the line and the committed profiles agree
  R=${ROUND:-r06}
  step prof 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra --no-exact --no-roofline-replays --no-aql
  python3 tools/trace_steps.py "$O/prof" "$O/prof.log" > "$O/step_spans.json"
  cp "$O/prof/run_kernel_stats.csv" "profiles/${R}_bench_rocprofv3_kernel_stats.csv"
  cp "$O/step_spans.json" "profiles/${R}_bench_rocprofv3_step_spans.json"
  step bench 480 python bench.py
  tail -1 "$O/bench.log" | cut -c1-400
fi
if has pmc; then     # decode GEMV HBM bytes: one counter per pass (gfx950: FETCH_SIZE is half the streamed bytes)
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_$c 300 rocprofv3 --pmc $c -d "$O/pmc/$c" -o run --output-format csv -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prefill --no-extra --no-exact --no-roofline-replays \
        --decode launches ${BENCH_ARGS:-}
  done
  python3 tools/pmc_summary.py "$O/pmc" > "$O/gemv_pmc_traffic.json" && cat "$O/gemv_pmc_traffic.json" | cut -c1-400
fi
if has gpmc; then    # prefill GEMM counters, k_gemm9 at 4096 x 4096 x 512 (tools/gemm_one.py)
  i=0
  IFS='|' read -ra sets <<< "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA|SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU|FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE SQ_INSTS_SALU"
  for c in "${sets[@]}"; do
    i=$((i+1))
    step gpmc_$i 60 rocprofv3 --pmc $c -d "$O/gpmc/p$i" -o run --output-format csv -- python3 tools/gemm_one.py
  done
fi
if has aql; then     # host cost per dispatch: hipLaunchKernelGGL vs a raw AQL packet on an own HSA queue (verdict r5 item 3)
  step aql 120 ./tools/aql_dispatch_cost tools/aql_kernel.hsaco
  cat "$O/aql.log"
fi
if has pchain; then  # prefill chain A/B (fixed x, dependent calls, chain with k_prep9_x, chain with epilogue images)
  step pchain 300 python tools/prefill_chain_ab.py ${PCHAIN_ROUNDS:-4}
  tail -1 "$O/pchain.log" | cut -c1-400
  for m in chain_fold chain_prep; do   # per-kernel durations of each chain form
    step pchain_$m 300 rocprofv3 --kernel-trace --stats -d "$O/$m" -o run --output-format csv -- \
        python3 tools/prefill_chain_ab.py 1 $m
  done
fi
if has mall; then    # GEMV per launch with HBM-streamed vs Infinity-Cache-resident weights (tools/mall_probe.py)
  step mall 300 python tools/mall_probe.py
  tail -1 "$O/mall.log" | cut -c1-600
fi
if has e2e; then     # the hook path end to end: the reference llama.cpp at full offload, LLaMA-7B shape
  step e2e 700 python tools/e2e_llama.py --decode 128 --modes fast,exact --out "$O/e2e_7b.json" ${E2E_ARGS:-}
fi
if has e2e_pad; then # the token time against a padded per-launch host cost (verdict r5 item 3: does submission bind?)
  step e2e_pad 900 python tools/e2e_llama.py --decode 64 --no-cpu \
      --modes fast,fast-pad1000,fast-pad2000,fast-pad3000,fast,fast-pad1000,fast-pad2000,fast-pad3000 --out "$O/e2e_pad.json"
  python3 -c "import json; r=json.load(open('$O/e2e_pad.json')); print({k: v['decode_tok_s'] for k, v in r.items() if k.startswith('offload')})"
fi
if has e2e_aql; then # launch mode 3 (own AQL queue) against eager launches, interleaved
  step e2e_aql 900 python tools/e2e_llama.py --decode 128 --no-cpu \
      --modes fast,fast-aql,fast,fast-aql,exact,exact-aql --out "$O/e2e_aql.json"
  python3 -c "import json; r=json.load(open('$O/e2e_aql.json')); print({k: (v['decode_tok_s'], v.get('backend_host_ms_per_eval'), v.get('aql_per_eval')) for k, v in r.items() if k.startswith('offload')})"
fi
if has e2e_ab; then  # the in-tree library against variants/libggml_hip_$VARIANT.so, separate processes, interleaved
  v=${VARIANT:-base}
  for i in 1 2; do
    step e2e_ab_base_$i 700 python tools/e2e_llama.py --decode 128 --no-cpu --modes ${AB_MODES:-fast} --out "$O/e2e_ab_base_$i.json"
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so step e2e_ab_${v}_$i 700 python tools/e2e_llama.py --decode 128 --no-cpu \
        --modes ${AB_MODES:-fast} --out "$O/e2e_ab_${v}_$i.json"
  done
  python3 -c "
import json, glob
for f in sorted(glob.glob('$O/e2e_ab_*.json')):
    r = json.load(open(f)); print(f.split('/')[-1], {k: v['decode_tok_s'] for k, v in r.items() if k.startswith('offload')})"
fi
if has e2e_kstats; then  # e2e decode kernel durations, in-tree library and the variant (rocprofv3 kernel trace)
  v=${VARIANT:-base}
  step e2e_ks_base 600 rocprofv3 --kernel-trace --stats -d "$O/ks_base" -o run --output-format csv -- \
      python3 tools/e2e_llama.py --decode 48 --no-cpu --modes fast
  GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so step e2e_ks_$v 600 rocprofv3 --kernel-trace --stats -d "$O/ks_$v" -o run \
      --output-format csv -- python3 tools/e2e_llama.py --decode 48 --no-cpu --modes fast
fi
if has kab; then      # decode GEMV launch times (tools/gemv_epi_ab.py), in-tree library vs variants/libggml_hip_$VARIANT.so
  v=${VARIANT:-base}
  for i in 1 2; do
    step kab_base_$i 300 python tools/gemv_epi_ab.py 200 2
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so step kab_${v}_$i 300 python tools/gemv_epi_ab.py 200 2
  done
  for f in "$O"/kab_*.log; do echo "## $f"; grep " us$" "$f"; done
fi
if has e2e_variant; then
  # a variant library through GGML_HIP_LIB, then the reference llama.cpp through the shim (the round-5 abort at
  # teardown): the process must exit 0 after llama_free / llama_free_model, with ONE libggml_hip mapped
  v=${VARIANT:-base}
  [ -f "variants/libggml_hip_$v.so" ] || { echo "variants/libggml_hip_$v.so missing: build it with tools/build_variant.sh"; exit 2; }
  GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so step e2e_variant 700 python tools/e2e_llama.py --decode 128 --no-cpu \
      --modes fast --maps --out "$O/e2e_variant_$v.json"
  python3 -c "import json; r=json.load(open('$O/e2e_variant_$v.json')); print('maps', r.get('libggml_hip_mapped'), 'tok/s', r['offload_fast']['decode_tok_s'])"
fi
exit 0
