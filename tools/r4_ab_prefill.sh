#!/bin/bash
# Interleaved A/B of whole-library variants on the bench prefill line (4 layers, sibling groups, fp6
# weight images): TOP/s and ms per layer.  LIBS="p9t1 p9t4" (variants/) or ENVS="b1:GGML_HIP_PREP9_BPW=1 ..."
# (settings of the in-tree library) ROUNDS=2
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
    env ${envs//,/ } GGML_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu \
        --no-exact --no-extra > gpurun_out/ab/pre_$v.$r.log 2> gpurun_out/ab/pre_$v.$r.err || { echo "$v rc=$?"; tail -5 gpurun_out/ab/pre_$v.$r.err; exit 1; }
    python - "$v" gpurun_out/ab/pre_$v.$r.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
p = r["prefill"]
print(f"{sys.argv[1]:8s} prefill {p['TOPs']} TOP/s {p['ms_per_layer']} ms/layer | decode {r['value']}", flush=True)
PY
  done
done
