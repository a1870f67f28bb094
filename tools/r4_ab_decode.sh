#!/bin/bash
# Interleaved A/B on the decode lines: the LLaMA-7B headline (per-shape launch times) and the other
# configs (13B, Falcon-7B, NeoX-20B).  Variants are whole libraries (LIBS="xwf0 xwf1", variants/) or
# environment settings of the in-tree library (ENVS="r3:GGML_HIP_GEMV_ROWMAX=3 r6:GGML_HIP_GEMV_ROWMAX=6").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS $ENVS; do
    case $v in
      *:*) name=${v%%:*}; envs=${v#*:}; lib=$PWD/llama.cpp-q_4_0_amd/libggml_hip.so ;;
      *) name=$v; envs=""; lib=$PWD/variants/libggml_hip_$v.so ;;
    esac
    v=$name
    env ${envs//,/ } GGML_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu \
        --no-prefill --no-exact > gpurun_out/ab/dec_$v.$r.log 2> gpurun_out/ab/dec_$v.$r.err || { echo "$v rc=$?"; tail -5 gpurun_out/ab/dec_$v.$r.err; exit 1; }
    python - "$v" gpurun_out/ab/dec_$v.$r.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ps = r["roofline"]["per_shape"]
oc = " ".join(f"{c['config'].split()[0]}={c['tok_s']}" for c in r.get("other_configs", []))
print(f"{sys.argv[1]:8s} {r['value']} tok/s frac {r['roofline']['frac']} |", " ".join(f"{k.split('->')[1]}={v['us']}" for k, v in ps.items()), "|", oc, flush=True)
PY
  done
done
