#!/bin/bash
# Interleaved A/B of whole-library variants (variants/libggml_hip_NAME.so, tools/build_variant.sh):
# decode headline with per-shape launch times, and (PREFILL=1) the bench's 512-token prefill line.
#   LIBS="base g9o1" ROUNDS=2 PREFILL=1 bash tools/r5_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
pf="--no-prefill"; [ -n "$PREFILL" ] && pf=""
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu \
        $pf --no-exact --no-extra > gpurun_out/ab/ab_$v.$r.log 2> gpurun_out/ab/ab_$v.$r.err || { echo "$v rc=$?"; tail -5 gpurun_out/ab/ab_$v.$r.err; exit 1; }
    python - "$v" gpurun_out/ab/ab_$v.$r.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ps = r["roofline"]["per_shape"]
pf = r.get("prefill")
pre = f"| prefill {pf['TOPs']} TOP/s {pf['ms_per_layer']} ms/layer" if pf else ""
print(f"{sys.argv[1]:8s} {r['value']} tok/s frac {r['roofline']['frac']} |", " ".join(f"{k.split('->')[1]}={v['us']}" for k, v in ps.items()), pre, flush=True)
PY
  done
done
