#!/bin/bash
# A/B of engine variant libraries (tools/build_variant.sh FILE=q4_0_engine NAME -D...): the engine_stamps summary
# of each, the in-tree library first.  O=gpurun_out/... VARIANTS="nc4 nc12" bash tools/engine_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/r06/ab}
mkdir -p "$O"
timeout -k 10 300 python tools/engine_stamps.py 32 > "$O/intree.json" 2> "$O/intree.err" || { echo "intree rc=$?"; tail -5 "$O/intree.err"; exit 1; }
python3 -c "import json; d=json.load(open('$O/intree.json')); print('intree', {k: v for k, v in d.items() if k.startswith('engine_diag') or k in ('launches_ms', 'per_layer_us_from_task_ends')})"
for v in ${VARIANTS}; do
  GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 300 python tools/engine_stamps.py 32 > "$O/$v.json" 2> "$O/$v.err" || { echo "$v rc=$?"; tail -5 "$O/$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', {k: v for k, v in d.items() if k.startswith('engine_diag') or k in ('launches_ms', 'per_layer_us_from_task_ends')})"
done
