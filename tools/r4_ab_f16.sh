#!/bin/bash
# A/B of the fast-mode f16 MFMA attention kernel variants (variants/libggml_hip_<name>.so) on the 500-token
# prompt shapes (tools/f16_mm_one.py): rocprofv3 kernel averages per shape.  LIBS="fmbase fmu1 fmu2 fmu4"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    rm -rf gpurun_out/ab/f16_$v.$r
    GGML_HIP_LIB=$PWD/variants/libggml_hip_$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ab/f16_$v.$r -o run \
        --output-format csv -- python3 tools/f16_mm_one.py > gpurun_out/ab/f16_$v.$r.log 2>&1 || { echo "$v rc=$?"; exit 1; }
    python3 - "$v" gpurun_out/ab/f16_$v.$r <<'PY'
import csv, glob, sys, statistics
f = glob.glob(sys.argv[2] + "/**/*kernel_trace.csv", recursive=True)[0]
by = {}
for r in csv.DictReader(open(f)):
    if "mul_mat_f16" in r["Kernel_Name"]:
        k = r["Grid_Size_X"] + "x" + r["Grid_Size_Y"]       # KQ and KQV differ in their grids
        by.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[1], " ".join(f"{k}: med {statistics.median(v):.2f} us" for k, v in sorted(by.items())), flush=True)
PY
  done
done
